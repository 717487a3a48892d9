#!/usr/bin/env python3
"""Interleaved A/B of tuning variants of the run-time compiled m = 6 butterfly
kernel, in ONE process (cdna_hip_programming.md §5.4 rule 24).

Each variant is a CVD_JIT_DEFINES string (e.g. "-DCVD_K1B_WAVES=5"); a fresh
model is created and uploaded per variant with that string in the
environment, so each gets its own compiled kernel (cvd_rtc.cpp keys its cache
by the defines).  One batch of streams per p is generated once; then
rounds x variants detector launches are timed with HIP events on the launch
stream, and every variant's per-trial sums must equal the first variant's.

usage: python profiles/ab_k1b.py --variant= --variant=-DCVD_K1B_WAVES=5 --p 0.01 0.1
       (host-side settings after a ';': --variant=";CVD_FILTER_SCALE=-1"; they are set at model
       build and around every launch of the variant, e.g. --variant=";CVD_WALK=0")
prints one JSON line per p: per-variant launch times (ms), medians and mins.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", action="append", dest="variants", default=None,
                    help="CVD_JIT_DEFINES of one variant, as --variant=-DX=1 (empty: the default kernel)")
    ap.add_argument("--p", type=float, nargs="+", default=[0.01, 0.1])
    ap.add_argument("--trials", type=int, default=655_360,
                    help="trials per launch (655,360 = 5 rounds at 4 waves/SIMD, 4 rounds at 5)")
    ap.add_argument("--N", type=int, default=100_000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--out", default=None, help="append the JSON lines to this file")
    ap.add_argument("--no-check", action="store_true",
                    help="ablation variants (-DCVD_ABL=...): time only, sums are expected to differ")
    a = ap.parse_args()
    a.variants = a.variants or [""]
    pkg = load_package()
    cc = pkg.CONFIG_CODES["m6"]
    det = pkg.Detector(1, 2, 6, cc["gen1"], device=0)
    g1, g2 = pkg.Code(cc["gen1"], 6, 1, 2), pkg.Code(cc["gen2"], 6, 1, 2)
    B, N = a.trials, a.N
    r = det.stream_buffer(N, 2 * B)
    stream = torch.cuda.current_stream()
    for p in a.p:
        tag = pkg.grid_tag(N, p)
        det.generate(g1, N, p, a.seed, tag, 0, 2, B, out=r, q0=0, pitch=2 * B)
        det.generate(g2, N, p, a.seed, tag, 1, 2, B, out=r, q0=B, pitch=2 * B)
        models = []
        envs_of = {}
        for v in a.variants:
            # a variant is JIT defines, optionally followed by ";VAR=value" host settings
            defs, *envs = v.split(";")
            envs_of[v] = [e.split("=", 1) for e in envs]
            os.environ["CVD_JIT_DEFINES"] = defs
            for e in envs:
                k_, v_ = e.split("=", 1)
                os.environ[k_] = v_
            models.append(pkg.Model(det.dec, p, None, 200, 1.0, a.seed).upload(0))
            for e in envs:
                os.environ.pop(e.split("=", 1)[0], None)
        os.environ.pop("CVD_JIT_DEFINES", None)
        kernels = [pkg.KERNEL_NAMES[mod.info()["explicit_kernel"]] for mod in models]
        def launch_env(v, on):
            for k_, v_ in envs_of[v]:
                if on:
                    os.environ[k_] = v_
                else:
                    os.environ.pop(k_, None)

        ref = None
        for v, mod in zip(a.variants, models):   # correctness: identical sums for every variant
            sums = torch.empty((2 * B, 2), dtype=torch.float64, device=det.device)
            launch_env(v, True)
            det.detect(mod, r, N, 2 * B, B, sums=sums)
            launch_env(v, False)
            s = sums.cpu().numpy()
            if ref is None:
                ref = s
            elif not a.no_check and not np.array_equal(s, ref):
                raise RuntimeError(f"variant {v!r}: sums differ from variant {a.variants[0]!r}")
            del sums
        times = {v: [] for v in a.variants}
        counts = torch.zeros(2, dtype=torch.int64, device=det.device)
        for _ in range(a.rounds):
            for v, mod in zip(a.variants, models):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                launch_env(v, True)
                e0.record(stream)
                det.detect(mod, r, N, 2 * B, B, counts=counts, stream=stream)
                e1.record(stream)
                launch_env(v, False)
                e1.synchronize()
                times[v].append(e0.elapsed_time(e1))
        line = {"p": p, "trials": B, "N": N, "kernels": kernels, "ms": times,
                "median": {v: float(np.median(t)) for v, t in times.items()},
                "min": {v: float(np.min(t)) for v, t in times.items()}}
        print(json.dumps(line), flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(json.dumps(line) + "\n")
        del models


if __name__ == "__main__":
    main()
