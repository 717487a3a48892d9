"""Host->HBM copy rate of received streams, for the PCIe-inclusive note in DESIGN.md.

The bench generates its streams on the device (Philox spec, D1), so its `value` never
crosses PCIe. A caller that instead hands cvd_detect host-resident streams must copy
them first: at N = 1e5, rate 1/2, one trial is two sequences of 6,250 u32 words
(50,000 B). This times pinned-host -> device copies of that layout and prints one
JSON line with the copy rate in trials/s.

    python profiles/pcie_h2d.py [--trials 131072] [--reps 5]
"""
import argparse
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=131072)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--N", type=int, default=100000)
    a = ap.parse_args()
    words = -(-a.N // 16)                      # n = 2: 16 steps per u32 word
    nbytes = a.trials * 2 * words * 4          # H1 + H2 sequence per trial
    host = torch.empty(nbytes // 4, dtype=torch.int32, pin_memory=True)
    host.fill_(0x5A5A5A5A)
    dev = torch.empty_like(host, device="cuda:0")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        dev.copy_(host, non_blocking=True)     # warm-up
        s.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            dev.copy_(host, non_blocking=True)
        e1.record(s)
        e1.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    print(json.dumps({"what": "pinned H2D copy of received streams", "N": a.N,
                      "trials": a.trials, "bytes_per_copy": nbytes,
                      "ms_per_copy": ms, "GB_per_s": nbytes / ms / 1e6,
                      "trials_per_s": a.trials / ms * 1e3}))


if __name__ == "__main__":
    main()
