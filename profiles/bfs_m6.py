#!/usr/bin/env python3
"""§8(f) row 2: the state count S of the m = 6 headline decoder (133,171) by the GPU
BFS (cvd_enumerate_device), or a certified lower bound with per-level sizes when the
search passes the device memory (or the time budget, CVD_BFS_SECONDS).

  CVD_BFS_VERBOSE=1 python profiles/bfs_m6.py gpurun_out/bfs_m6.json [mem_GiB]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
out_path = sys.argv[1]
mem = int(float(sys.argv[2]) * (1 << 30)) if len(sys.argv) > 2 else 0
res = {}
for name, cc in (("m4_2335", {"gen1": [[[1, 0, 0, 1, 1]], [[1, 1, 1, 0, 1]]], "m": 4}),
                 ("m5_53_75", {"gen1": [[[1, 0, 1, 0, 1, 1]], [[1, 1, 1, 1, 0, 1]]], "m": 5}),
                 ("m6_133_171", {"gen1": pkg.CONFIG_CODES["m6"]["gen1"], "m": 6})):
    t0 = time.perf_counter()
    r = pkg.enumerate_states_device(cc["gen1"], cc["m"], 1, 2, device=0, mem_bytes=mem)
    r["seconds"] = time.perf_counter() - t0
    r["levels"] = len(r["level_sizes"])
    res[name] = r
    print(name, {k: v for k, v in r.items() if k != "level_sizes"}, flush=True)
    json.dump(res, open(out_path, "w"), indent=1)
