#!/bin/bash
# round 3: lockstep kernel at 4 / 3 / 2 waves per SIMD (LDS padding lowers the blocks per CU)
set -uo pipefail
O=gpurun_out/r03q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u profiles/ab_k1b.py --variant=";CVD_WALK=0" --variant="-DCVD_K1B_LDS_PAD=15000;CVD_WALK=0" \
  --variant="-DCVD_K1B_LDS_PAD=20000;CVD_WALK=0" --p 0.01 0.1 \
  --rounds 2 --out $O/ab_occ.jsonl > $O/ab_occ.log 2>&1 || { echo "AB OCC FAILED"; tail -20 $O/ab_occ.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r03q/ab_occ.jsonl"):
    d = json.loads(l); print(d["p"], {k: round(v, 1) for k, v in d["median"].items()})
PY
