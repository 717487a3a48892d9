"""Turn a profiles/collect.sh output directory (gpurun_out/...) into the
committed evidence: profiles/<name>/ (rocprofv3 kernel stats, trace and PMC
CSVs trimmed to the detector and generator) and the per-launch PMC summary,
which bench.py reads for roofline.traffic (profiles/pmc_<detector>_<config>.json).

  python profiles/summarize.py gpurun_out/prof r01d_m6
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def is_det(name):
    return "detect" in name or "k1b" in name or "parity_kernel" in name


def is_gen(name):
    return "gen_" in name


def main(src, name):
    dst = os.path.join(ROOT, "profiles", name)
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))[0]
    shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    trace = glob.glob(os.path.join(src, "trace", "*kernel_trace.csv"))[0]
    rows = [r for r in csv.DictReader(open(trace)) if is_det(r["Kernel_Name"]) or is_gen(r["Kernel_Name"])]
    with open(os.path.join(dst, "kernel_trace.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)
    bench = json.load(open(os.path.join(src, "bench_trace.json")))
    json.dump(bench, open(os.path.join(dst, "bench_under_rocprof.json"), "w"), indent=1)
    agg, cnt = {}, {}
    for i, f in enumerate(sorted(glob.glob(os.path.join(src, "pmc*", "*counter_collection.csv")))):
        keep = [r for r in csv.DictReader(open(f)) if is_det(r["Kernel_Name"]) or is_gen(r["Kernel_Name"])]
        tag = os.path.basename(os.path.dirname(f))
        with open(os.path.join(dst, f"{tag}.csv"), "w", newline="") as g:
            w = csv.DictWriter(g, fieldnames=list(keep[0].keys()))
            w.writeheader()
            w.writerows(keep)
        for r in keep:
            if is_det(r["Kernel_Name"]):
                k = r["Counter_Name"]
                agg[k] = agg.get(k, 0.0) + float(r["Counter_Value"])
                cnt[k] = cnt.get(k, 0) + 1
    per = {k: agg[k] / cnt[k] for k in agg}
    cfg = bench["config"]
    B, N = cfg["trials_per_step_per_gpu"], cfg["N"]
    waves = per.get("SQ_WAVES", 2 * B / 64)
    kernel_cycles = per.get("GRBM_GUI_ACTIVE", 0.0) / 8   # GRBM_GUI_ACTIVE sums the 8 XCDs
    out = {
        "kernel": bench["roofline"]["kernel"],
        "workload": f"bench.py --steps 2 --warmup 0 (p = 0.01, 0.02), {B} trials x 2 sequences, N = {N}",
        "source": "rocprofv3 --pmc, one counter group per pass (profiles/collect.sh), averaged per detector launch",
        "FETCH_SIZE_kB_per_launch": per.get("FETCH_SIZE"),
        "WRITE_SIZE_kB_per_launch": per.get("WRITE_SIZE"),
        "detector_fetch_bytes_per_launch_raw": per.get("FETCH_SIZE", 0.0) * 1024,
        # The guide's x2 (FETCH_SIZE = half of a 16-B/lane streaming read) applies to the
        # stream chunks only: they are the algorithmic bytes, read once as 16-B lane loads,
        # so they appear as algorithmic / 2 in the raw count.  The rest (filter words,
        # directory lines, row records: 8-128 B random reads, uncalibrated) is taken raw.
        "detector_fetch_bytes_per_launch": per.get("FETCH_SIZE", 0.0) * 1024 + min(
            per.get("FETCH_SIZE", 0.0) * 1024, bench["roofline"]["algorithmic_bytes_per_launch"] / 2),
        "traffic_basis": "rocprofv3 FETCH_SIZE; the 16-B/lane stream reads x2 (MI355X_MICROARCH.md), the random reads raw",
        "correction": "x2 on the stream part only (algorithmic bytes / 2 of the raw count: 16-B/lane chunk loads, read "
                      "once); the row-table traffic is 8-128 B random accesses, which the guide leaves uncalibrated, "
                      "taken raw",
        "algorithmic_bytes_per_launch": bench["roofline"]["algorithmic_bytes_per_launch"],
        "SQ_INSTS_VALU_per_launch": per.get("SQ_INSTS_VALU"),
        "VALU_insts_per_wave_step": per.get("SQ_INSTS_VALU", 0.0) / (waves * N),
        "SALU_insts_per_wave_step": per.get("SQ_INSTS_SALU", 0.0) / (waves * N),
        "VMEM_RD_insts_per_wave_step": per.get("SQ_INSTS_VMEM_RD", 0.0) / (waves * N),
        "SQ_WAVES": waves,
        "GRBM_GUI_ACTIVE": per.get("GRBM_GUI_ACTIVE"),
        "kernel_cycles": kernel_cycles,
        # VALU issue capacity: 1024 SIMDs, one wave64 instruction per 2 cycles (plain VOP2
        # add/sub/logic/16-bit) or 4 cycles (VOP3/VOP3P/shifts: the packed ACS ops),
        # measured on MI355X (.scratch microbenchmarks); the hot loop averages
        # ~3.5 issue cycles per VALU instruction (static mix of the JIT kernel)
        "valu_issue_frac_est": per.get("SQ_INSTS_VALU", 0.0) * 3.5 / (1024 * max(1.0, kernel_cycles)),
        "wait_inst_any_frac_of_wave_cycles": per.get("SQ_WAIT_INST_ANY", 0.0) / max(1.0, per.get("SQ_WAVE_CYCLES", 1.0)),
        "active_valu_frac_of_wave_cycles": per.get("SQ_ACTIVE_INST_VALU", 0.0) / max(1.0, per.get("SQ_WAVE_CYCLES", 1.0)),
        "counters_per_launch": per,
        "config": cfg.get("name", "m6"),
        "detector": cfg.get("detector", "markov"),
        "batch": B,
        "N": N,
    }
    # cycle-weighted VALU issue fraction: the step loop's opcode mix (static ISA of
    # the kernel this tree builds, profiles/isa_breakdown.py) priced with the measured
    # issue cost per class (profiles/valu_issue_cycles.json), times the dynamic
    # instruction count, over the launch's SIMD-cycles
    if out["detector"] == "markov" and "k1b" in out["kernel"]:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import isa_breakdown
        import valu_model
        import tempfile
        with tempfile.TemporaryDirectory() as d:
            lines = isa_breakdown.build_isa(out["config"], [], os.path.join(d, "k.s"))
        mix = {}
        for _name, ins in isa_breakdown.blocks(isa_breakdown.main_loop(lines)):
            for x in ins:
                if x.startswith("v_"):
                    mix[x.split()[0]] = mix.get(x.split()[0], 0) + 0.25    # 4 steps per loop trip
        cyc, by = valu_model.load_cycles()
        avg, by_class = valu_model.weighted_cycles(mix, cyc)
        out["valu_cycles_per_inst"] = avg
        out["valu_cycles_source"] = ("static opcode mix of the step loop (profiles/isa_breakdown.py) x measured "
                                     "issue cost per class (profiles/valu_issue_cycles.json)")
        out["valu_mix_by_class_per_step"] = by_class
        out["valu_issue_cycle_frac"] = per.get("SQ_INSTS_VALU", 0.0) * avg / (1024 * max(1.0, kernel_cycles))
    fn = f"pmc_{out['detector']}_{out['config']}.json"
    json.dump(out, open(os.path.join(ROOT, "profiles", fn), "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "counters_per_launch"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
