#!/bin/bash
# round 3: CVD_K1B_CMPX in the lockstep body only (walk ACS steps keep the xor compare);
# walk schedule amin 2 / 4 with wmin 44 / 48
set -uo pipefail
O=gpurun_out/r03p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u profiles/ab_k1b.py --variant= --variant=-DCVD_K1B_CMPX=1 \
  "--variant=-DCVD_K1B_CMPX=1 -DCVD_K1B_CMPX_WALK=0" --p 0.01 0.02 0.1 \
  --rounds 3 --out $O/ab_cmpx_walk.jsonl > $O/ab_cmpx_walk.log 2>&1 || { echo "AB CMPX FAILED"; tail -20 $O/ab_cmpx_walk.log; exit 1; }
timeout -k 10 400 python -u profiles/ab_k1b.py --variant= --variant=";CVD_WALK_AMIN=2" --variant=";CVD_WALK_AMIN=4" \
  --variant=";CVD_WALK_AMIN=4;CVD_WALK_WMIN=44" --variant=";CVD_WALK_AMIN=2;CVD_WALK_WMIN=44" --p 0.01 0.02 \
  --rounds 3 --out $O/ab_sched2.jsonl > $O/ab_sched2.log 2>&1 || { echo "AB SCHED FAILED"; tail -20 $O/ab_sched2.log; exit 1; }
python3 - <<'PY'
import json
for f in ["gpurun_out/r03p/ab_cmpx_walk.jsonl", "gpurun_out/r03p/ab_sched2.jsonl"]:
    for l in open(f):
        d = json.loads(l); print(d["p"], {k: round(v, 1) for k, v in d["median"].items()})
PY
echo ALL DONE
