#!/bin/bash
# round 3 ablation (timing only, sums differ): waves of H2 sequences skip their Bloom-filter
# read (CVD_ABL & 64), in walk mode and in lockstep -- how much do the per-step random L2
# reads of the H2 waves cost?
set -uo pipefail
O=gpurun_out/r03w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u profiles/ab_k1b.py --no-check --variant= --variant=-DCVD_ABL=64 \
  --variant=";CVD_WALK=0" --variant="-DCVD_ABL=64;CVD_WALK=0" --p 0.01 0.02 0.1 \
  --rounds 2 --out $O/ab_abl64.jsonl > $O/ab_abl64.log 2>&1 || { echo "AB FAILED"; tail -20 $O/ab_abl64.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r03w/ab_abl64.jsonl"):
    d = json.loads(l); print(d["p"], {k: round(v, 1) for k, v in d["median"].items()})
PY
