#!/usr/bin/env python3
"""Benchmark: Monte-Carlo trials/s of the relative-Viterbi-metric detector.

BASELINE.json metric: "MC trials/sec at N=1e5, rate-1/2 m=6 pair, 1/2/4/8 GPUs;
Pd match vs CPU".  Workload (configs[2]): the m = 6 pair (133,171) vs (171,133),
N = 1e5, p swept over {0.01, 0.02, 0.05, 0.10, 0.15, 0.20}.

One trial = one H1 plus one H2 sequence of length N (one iteration of
Pd_plotter.py:210-223).  One step = one batch of `--batch` trials per GPU at
one p of the sweep (step s uses p_grid[s % 6]): the generator kernel writes the
batch's BSC-noised received streams to HBM (encoder + Philox noise, two
launches: H1 with G1, H2 with G2), then the detector kernel reads them
(Eq. 4-5 recursion for all 2^n received words, T_ref count, hashed P̂1 row
lookup, fp64 log-likelihood sums, decisions, counts).  Both kernels are inside
the timed region; learning P̂1 (host setup, once per p) is not.

Multi-GPU (torchrun): one process per GPU, rank r takes its own global trial
ids every step (weak scaling); the success counts are reduced with one RCCL
all_reduce at the end of the timed region.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402

METRIC = "MC trials/sec at N=1e5, rate-1/2 m=6 pair, 1/2/4/8 GPUs; Pd match vs CPU"
P_GRID = [0.01, 0.02, 0.05, 0.10, 0.15, 0.20]
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, one GPU per rank); gloo only to rehearse the multi-rank path")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="m6", choices=["m6", "m2", "r23_m4"])
    ap.add_argument("--N", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None, help="trials per GPU per step")
    ap.add_argument("--learn-len", type=int, default=1_000_000,
                    help="P̂1 learning chain length for non-enumerable codes")
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--p", type=float, default=None, help="diagnostic: run one p instead of the sweep")
    ap.add_argument("--detector", default="markov", choices=["markov", "parity"],
                    help="markov: the relative-Viterbi-metric detector (headline); parity: the "
                         "parity-template baseline of comp_parity.py on the same streams")
    ap.add_argument("--gamma", type=float, default=0.6, help="parity baseline threshold (comp_parity.py:151)")
    ap.add_argument("--overlap", type=int, default=-1,
                    help="generate the next batch on a second stream while the detector runs "
                         "(-1: auto = on for the table automaton, where it measured faster)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the C oracle port (rank 0, N=1)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--pmc-traffic", default=None,
                    help="per-launch detector FETCH_SIZE summary of a rocprofv3 --pmc pass "
                         "(profiles/collect.sh + summarize.py; default profiles/pmc_<detector>_<config>.json); "
                         "used only when its config/batch/N match this run")
    return ap.parse_args()


def main():
    a = parse()
    pkg = load_package()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.dist_backend == "gloo" and os.environ.get("CVD_BENCH_ONE_DEVICE") == "1":
        local = 0   # rehearsal of the multi-rank path on a one-GPU box (RCCL needs one GPU per rank)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    cc = pkg.CONFIG_CODES[a.config]
    k, n, m = cc["k"], cc["n"], cc["m"]
    N = a.N if a.N is not None else {"m6": 100_000, "m2": 10_000, "r23_m4": 100_000}[a.config]
    p_grid = P_GRID if a.config != "m2" else [0.05]
    if a.p is not None:
        p_grid = [a.p]   # diagnostic: one grid point only (not the headline sweep)
    det = pkg.Detector(k, n, m, cc["gen1"], device=local)
    g1 = pkg.Code(cc["gen1"], m, k, n)
    g2 = pkg.Code(cc["gen2"], m, k, n)
    parity = a.detector == "parity"
    if parity:
        # parity-template baseline (comp_parity.py): template of G1, no learned model
        tpl = pkg.default_template(cc["gen1"], m)
        models, info = {}, {"kind": 0, "explicit_kernel": 0, "learn_len_eff": 0, "n_rows": 0}
    else:
        models = dict(zip(p_grid, det.prepare_models(p_grid, a.learn_len if m == 6 else None, 200, 1.0, a.seed)))
        info = models[p_grid[0]].info()
    # whole residency rounds: 4 waves/SIMD x 1024 SIMDs x 64 lanes = 262,144 sequences
    # (131,072 trials) per round.  m6: 20 rounds per launch (131 GB of streams) -- the
    # last round's uneven wave finish costs ~24 ms per launch, amortised over the rounds
    # (DESIGN.md "Launch size": 687k trials/s at 2 rounds, 735k at 10, 742k at 20)
    # m2: 2^22 trials (56.0M vs 52.3M trials/s at 2^20); r23_m4: 2^17 measured best
    B = a.batch or {"m6": 2_621_440, "m2": 4_194_304, "r23_m4": 131_072}[a.config]
    # double-buffered pipeline: the generator fills buffer (s+1)%2 on its own
    # stream while the detector reads buffer s%2 (both kernels of every timed
    # step run inside the timed region)
    if a.overlap < 0:
        a.overlap = int(not info["kind"])
    buf_bytes = det.words_per_seq(N) * 4 * 2 * B
    if a.overlap and 2 * buf_bytes > (120 << 30):
        a.overlap = 0                          # two batches would not leave HBM headroom
    nbuf = 2 if a.overlap else 1
    bufs = [det.stream_buffer(N, 2 * B) for _ in range(nbuf)]
    counts = torch.zeros((len(p_grid), 2), dtype=torch.int64, device=det.device)
    dstream = torch.cuda.current_stream()
    gstream = torch.cuda.Stream(device=det.device) if a.overlap else dstream

    def gen(s, ev=None):
        p = p_grid[s % len(p_grid)]
        tb = (s * world + rank) * B            # global trial ids of this rank's batch
        tag = pkg.grid_tag(N, p)
        r = bufs[s % nbuf]
        if ev is not None:
            ev[0].record(gstream)
        det.generate(g1, N, p, a.seed, tag, 2 * tb, 2, B, out=r, q0=0, pitch=2 * B, stream=gstream)
        det.generate(g2, N, p, a.seed, tag, 2 * tb + 1, 2, B, out=r, q0=B, pitch=2 * B, stream=gstream)
        if ev is not None:
            ev[1].record(gstream)

    def detect(s, ev=None):
        p = p_grid[s % len(p_grid)]
        if ev is not None:
            ev[2].record(dstream)
        if parity:
            pkg.parity_detect(bufs[s % nbuf], n, N, 2 * B, B, tpl, a.gamma, counts=counts[s % len(p_grid)],
                              stream=dstream)
        else:
            det.detect(models[p], bufs[s % nbuf], N, 2 * B, B, counts=counts[s % len(p_grid)], stream=dstream)
        if ev is not None:
            ev[3].record(dstream)

    def run(steps, base, events=None):
        if not a.overlap:
            for s in range(steps):
                ev = events[s] if events else None
                gen(base + s, ev)
                detect(base + s, ev)
            return
        done = [torch.cuda.Event() for _ in range(steps)]
        ready = [torch.cuda.Event() for _ in range(steps)]
        gen(base, events[0] if events else None)
        ready[0].record(gstream)
        for s in range(steps):
            dstream.wait_event(ready[s])
            detect(base + s, events[s] if events else None)
            done[s].record(dstream)
            if s + 1 < steps:
                if s >= 1:
                    gstream.wait_event(done[s - 1])   # buffer (s+1)%2 was read by detect(s-1)
                gen(base + s + 1, events[s + 1] if events else None)
                ready[s + 1].record(gstream)
        dstream.wait_stream(gstream)

    run(a.warmup, 10_000)
    counts.zero_()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(a.steps)]
    t0 = time.perf_counter()
    run(a.steps, 0, events)
    if dist:
        dist.all_reduce(counts)                # the one collective: success counts over RCCL
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=det.device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    gen_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in events]))
    det_each = [e[2].elapsed_time(e[3]) for e in events]
    det_ms = float(np.mean(det_each))

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    trials = a.steps * B * world
    value = trials / elapsed
    # roofline of the dominant kernel (detector): algorithmic bytes = the packed
    # received streams read once, 2 * ceil(N * n / 8) bytes per trial
    alg_bytes = B * 2 * ((N * n + 7) // 8)
    achieved = alg_bytes / (det_ms * 1e-3) / 1e9
    traffic, traffic_src, valu = None, None, None
    if a.pmc_traffic is None:
        a.pmc_traffic = os.path.join(ROOT, "profiles", f"pmc_{a.detector}_{a.config}.json")
    if a.pmc_traffic and os.path.exists(a.pmc_traffic):
        with open(a.pmc_traffic) as f:
            pmc = json.load(f)
        if (pmc.get("config"), pmc.get("batch"), pmc.get("N"), pmc.get("detector", "markov")) == \
                (a.config, B, N, a.detector):
            traffic = pmc.get("detector_fetch_bytes_per_launch")
            valu = {k: pmc.get(k) for k in ("VALU_insts_per_wave_step", "valu_issue_frac_est", "kernel")}
            traffic_src = os.path.relpath(a.pmc_traffic, ROOT) + " (rocprofv3 FETCH_SIZE x1024 x2, gfx950 correction)"
    c = counts.cpu().numpy()
    per_p = {str(p): {"Pd": float(c[i, 0]) / max(1, (a.steps // len(p_grid) + (i < a.steps % len(p_grid))) * B * world),
                      "h1_successes": int(c[i, 0]), "h2_successes": int(c[i, 1])}
             for i, p in enumerate(p_grid)}
    out = {
        "metric": (METRIC if a.config == "m6" and not parity
                   else f"MC trials/sec ({a.config}, N={N}{', parity-template baseline' if parity else ''})"),
        "value": value,
        "unit": "trials/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16x2 (metrics) + f64 (log-likelihood sums)",
        "data": "synthetic: Philox4x32-10 encoder inputs and BSC(p) flips (build spec), learned P̂1",
        "config": {"name": a.config, "detector": a.detector,
                   "workload": f"{a.config} pair {cc['gen1']} vs {cc['gen2']}, N={N}, p-sweep {p_grid}, "
                               f"one p per step", "N": N, "p_grid": p_grid,
                   "trials_per_step_per_gpu": B, "model": info["kind"] and "sparse(learned)" or "dense",
                   "learn_len": info["learn_len_eff"], "model_rows_p0": info["n_rows"],
                   "parallelism": f"dp{world} (trial sharding, one RCCL all_reduce of counts)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": ("parity_kernel (parity-template baseline, cvd_parity.hip)" if parity
                                else pkg.KERNEL_NAMES[info["explicit_kernel"]] if info["kind"]
                                else "detect_table_kernel (enumerated state automaton)"),
                     "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": alg_bytes, "avg_launch_ms": det_ms},
        "diagnostic": {"generator_ms_per_step": gen_ms, "detector_ms_per_step": det_ms,
                       "overlap": bool(a.overlap),
                       "seq_steps_per_s_detector": 2 * B * N / (det_ms * 1e-3),
                       "detector_ms_by_p": {str(p_grid[s % len(p_grid)]): det_each[s] for s in range(a.steps)},
                       "detector_ms_steps": det_each,
                       # the binding resource is VALU issue, not HBM: from the PMC summary
                       "valu_bound": valu,
                       "per_p": per_p},
    }
    if a.cpu_baseline and world == 1 and not parity:
        out["cpu_baseline"], cpu_check = cpu_baseline(cc, k, n, m, N, a.seed, a.learn_len, a.cpu_seconds)
        if 0.05 in models:
            out["pd_match_vs_cpu"] = pd_match(det, models[0.05], cc, N, a.seed, cpu_check)
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def cpu_baseline(cc, k, n, m, N, seed, learn_len, seconds):
    """The oracle's C port of the reference path (oracle/cvd_oracle.c), OpenMP over
    trials on this host's cores, on a bounded sample of the same workload."""
    from oracle import c_oracle as C
    threads = min(16, os.cpu_count() or 1)
    c1, c2 = C.Code(cc["gen1"], m, k, n), C.Code(cc["gen2"], m, k, n)
    p = 0.05
    mod = C.Model(c1, p, learn_len if m == 6 else None, 200, 1.0, seed)
    # calibrate with one trial per thread, then size the sample to ~`seconds`
    t0 = time.perf_counter()
    c_cal, s_cal = mod.run_trials(c1, c2, N, p, seed, 0, threads, sums=True, nthreads=threads)
    dt = time.perf_counter() - t0
    ntr = max(threads, int(threads * seconds / max(dt, 1e-6)) // threads * threads)
    t0 = time.perf_counter()
    c_smp, _ = mod.run_trials(c1, c2, N, p, seed, threads, threads + ntr, nthreads=threads)
    dt = time.perf_counter() - t0
    check = {"p": p, "trials": threads + ntr, "counts": [int(x) for x in c_cal + c_smp], "sums": s_cal}
    return {"value": ntr / dt, "unit": "trials/s", "cores": threads, "kind": "port",
            "sample": f"{ntr} trials (H1+H2, N={N}) at p={p}, C oracle (oracle/cvd_oracle.c), "
                      f"{threads} OpenMP threads, {dt:.1f} s",
            "seconds": dt}, check


def pd_match(det, model, cc, N, seed, check):
    """The metric's "Pd match vs CPU": the GPU path on the CPU sample's trial ids
    (same model, same streams) -- success counts equal, and the per-trial fp64
    log-likelihood sums of the calibration trials bit-identical.  Outside the
    timed region."""
    T, p = check["trials"], check["p"]
    got = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, seed, 0, T)["counts"].cpu().tolist()
    ncal = len(check["sums"])
    sums = det.run_trials(model, cc["gen1"], cc["gen2"], N, p, seed, 0, ncal, return_sums=True)["sums"]
    same_sums = bool(np.array_equal(sums, check["sums"]))
    return {"p": p, "trials": T, "gpu_counts": got, "cpu_counts": check["counts"],
            "pd_gpu": got[0] / T, "pd_cpu": check["counts"][0] / T,
            "sums_bit_exact_trials": ncal, "match": got == check["counts"] and same_sums}


if __name__ == "__main__":
    main()
