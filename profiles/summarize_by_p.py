"""Summarise a profiles/pmc_by_p.sh output directory into pmc_by_p.json:
detector (cvd_k1b_spec) counters per grid point, per wave-step and per launch.

  python profiles/summarize_by_p.py gpurun_out/pmcp profiles/<name>
"""
import csv
import glob
import json
import os
import sys


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    per_p = {}
    for d in sorted(glob.glob(os.path.join(src, "p*_g*"))):
        if not os.path.isdir(d):
            continue
        p = os.path.basename(d)[1:].rsplit("_g", 1)[0]
        e = per_p.setdefault(p, {"counters": {}})
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                if "k1b" in r["Kernel_Name"]:
                    e["counters"][r["Counter_Name"]] = e["counters"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        bj = d + ".json"
        if os.path.exists(bj):
            b = json.loads(open(bj).read().strip().splitlines()[-1])
            e["detector_ms"] = b["diagnostic"]["detector_ms_per_step"]
            e["N"] = b["config"]["N"]
            e["trials"] = b["config"]["trials_per_step_per_gpu"]
    for p, e in per_p.items():
        c, waves = e["counters"], 2 * e["trials"] / 64
        ws = waves * e["N"]
        e["valu_per_wave_step"] = c.get("SQ_INSTS_VALU", 0.0) / ws
        e["vmem_rd_per_wave_step"] = c.get("SQ_INSTS_VMEM_RD", 0.0) / ws
        e["fetch_size_GB_raw"] = c.get("FETCH_SIZE", 0.0) * 1024 / 1e9
        e["wait_any_frac_of_wave_cycles"] = c.get("SQ_WAIT_ANY", 0.0) / max(1.0, c.get("SQ_WAVE_CYCLES", 1.0))
    out = {"what": "cvd_k1b_spec PMC per grid point: bench.py --p P --steps 1 (one detector launch), one "
                   "rocprofv3 --pmc pass per counter group (profiles/pmc_by_p.sh)", "per_p": per_p}
    json.dump(out, open(os.path.join(dst, "pmc_by_p.json"), "w"), indent=1)
    for p, e in sorted(per_p.items(), key=lambda x: float(x[0])):
        print(p, round(e.get("detector_ms", 0)), round(e["valu_per_wave_step"], 1), round(e["vmem_rd_per_wave_step"], 2),
              round(e["fetch_size_GB_raw"], 1), round(e["wait_any_frac_of_wave_cycles"], 3))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
