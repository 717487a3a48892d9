#!/bin/bash
# round 3: log P̂1 of unvisited rows in a VGPR pair across the step loop (CVD_K1B_LPU_VGPR) A/B
set -uo pipefail
O=gpurun_out/r03v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u profiles/ab_k1b.py --variant= --variant=-DCVD_K1B_LPU_VGPR=1 --p 0.01 0.02 0.05 0.1 0.2 \
  --rounds 3 --out $O/ab_lpu.jsonl > $O/ab_lpu.log 2>&1 || { echo "AB FAILED"; tail -20 $O/ab_lpu.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r03v/ab_lpu.jsonl"):
    d = json.loads(l); print(d["p"], {k: round(v, 1) for k, v in d["median"].items()})
PY
