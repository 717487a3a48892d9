"""Generator-only driver for profiling gen_fast_kernel (rocprofv3 --pmc passes):
one code's received streams for a batch of sequences, timed with HIP events.
  python profiles/gen_only.py m2 [reps]        (GEN_ONLY_LIB=path: another libcvd.so)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib  # noqa: E402

pkg = importlib.import_module("detecting-convolutional-codes-via-markovian-statistics_amd")
if os.environ.get("GEN_ONLY_LIB"):   # A/B: another build of libcvd.so
    importlib.import_module("detecting-convolutional-codes-via-markovian-statistics_amd._lib").LIB_PATH = \
        os.environ["GEN_ONLY_LIB"]

CASES = {"m2": ("m2", 10_000, 1 << 22), "m6": ("m6", 100_000, 1 << 18), "r23_m4": ("r23_m4", 100_000, 1 << 18)}
name = sys.argv[1] if len(sys.argv) > 1 else "m2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
cfg, N, count = CASES[name]
cc = pkg.CONFIG_CODES[cfg]
k, n, m = cc["k"], cc["n"], cc["m"]
det = pkg.Detector(k, n, m, cc["gen1"], device=0)
out = det.stream_buffer(N, count)
for p in (0.0, 0.01, 0.05, 0.2):
    ms = []
    for r in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        det.generate(cc["gen1"], N, p, 1234, 5678, 0, 1, count, out=out)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    print(f"{name} N={N} count={count} p={p}: ms {min(ms):.3f}", flush=True)
