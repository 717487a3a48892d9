#!/bin/bash
# round 3: walk schedule on the final tree (LDS filter at p = 0.01): burst length and wmin
set -uo pipefail
O=gpurun_out/r03af
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u profiles/ab_k1b.py --variant= --variant=";CVD_WALK_BURST=5" --variant=";CVD_WALK_BURST=3" \
  --variant=";CVD_WALK_WMIN=40" --variant=";CVD_WALK_WMIN=44" --p 0.01 0.02 --rounds 2 \
  --out $O/ab_sched3.jsonl > $O/ab_sched3.log 2>&1 || { echo "AB FAILED"; tail -20 $O/ab_sched3.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r03af/ab_sched3.jsonl"):
    d = json.loads(l); print(d["p"], {k: round(v, 1) for k, v in d["median"].items()})
PY
