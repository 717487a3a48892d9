#!/bin/bash
# round 3: two-step walk records read only for the hottest K rows (others one step per load):
# does the records' cache footprint bound the walks?
set -uo pipefail
O=gpurun_out/r03aa
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u profiles/ab_k1b.py --trials 2621440 --variant= --variant=";CVD_T2_ROWS=8192" \
  --variant=";CVD_T2_ROWS=4096" --variant=";CVD_T2_ROWS=2048" --p 0.01 0.02 \
  --rounds 1 --out $O/ab_t2rows.jsonl > $O/ab_t2rows.log 2>&1 || { echo "AB FAILED"; tail -20 $O/ab_t2rows.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r03aa/ab_t2rows.jsonl"):
    d = json.loads(l); print(d["p"], {k: round(v, 1) for k, v in d["median"].items()})
PY
