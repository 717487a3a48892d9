"""What bounds the dense-table kernels: LDS-array occupancy and bank
conflicts beside VALU issue, from the two rocprofv3 --pmc passes of profiles/r04_lds_pmc.sh.

  python profiles/lds_bound.py gpurun_out/r04f      -> profiles/pmc_lds_<config>.json

Per launch (one dispatch of the detector kernel):
  lds_busy      = SQ_LDS_IDX_ACTIVE / CUs / kernel cycles (the LDS array's share of the
                  launch; SQ_LDS_IDX_ACTIVE counts LDS-array cycles summed over the CUs,
                  MI355X_MICROARCH.md LDS)
  conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles of lanes on one
                  bank with distinct addresses)
  valu_issue_2cyc = SQ_INSTS_VALU x 2 cycles / (SIMDs x kernel cycles)
  kernel cycles = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs)
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CUS, SIMDS = 256, 1024


def load(d, cfg):
    """counter -> mean per dispatch of the detector kernel (GRBM_GUI_ACTIVE is in both
    passes: averaged over them)"""
    vals, name = {}, None
    for f in sorted(glob.glob(os.path.join(d, f"{cfg}_pmc*", "*counter_collection.csv"))):
        per_disp = {}
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "table" not in k and "detect" not in k:
                continue
            name = k.split("(")[0].split("<")[0].strip()
            e = per_disp.setdefault(r["Dispatch_Id"], {})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for e in per_disp.values():
            for c, v in e.items():
                vals.setdefault(c, []).append(v)
    return name, {c: sum(v) / len(v) for c, v in vals.items()}


def main(d):
    for cfg in ("m2", "r23_m4"):
        kern, c = load(d, cfg)
        if kern:
            kc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8
            out = {"config": cfg, "kernel": kern, "source": f"rocprofv3 --pmc, profiles/r04_lds_pmc.sh ({os.path.basename(d)})",
                   "counters_per_launch": c,
                   "kernel_cycles": kc,
                   "lds_busy": c["SQ_LDS_IDX_ACTIVE"] / CUS / kc,
                   "lds_conflict_frac": c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"],
                   "lds_insts_per_wave_cycle_kernel": c["SQ_INSTS_LDS"] / SIMDS / kc,
                   "lds_array_cycles_per_lds_inst": c["SQ_LDS_IDX_ACTIVE"] / c["SQ_INSTS_LDS"],
                   "valu_issue_2cyc": c["SQ_INSTS_VALU"] * 2 / (SIMDS * kc),
                   "bound": "lds"}
            fn = os.path.join(ROOT, "profiles", f"pmc_lds_{cfg}.json")
            json.dump(out, open(fn, "w"), indent=1)
            print(cfg, kern, {k: round(v, 3) for k, v in out.items() if isinstance(v, float)})


if __name__ == "__main__":
    main(sys.argv[1])
