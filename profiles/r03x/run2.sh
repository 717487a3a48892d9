#!/bin/bash
# round 3: which part of the LDS-filter variant costs: block size (256 / 512 / 1,024) with the
# global filter, and the LDS filter at 512 threads (64 KiB filter) and 1,024 (128 KiB)
set -uo pipefail
O=gpurun_out/r03x2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u profiles/ab_k1b.py --variant=";CVD_NO_LDSF=1" --variant=";CVD_NO_LDSF=1;CVD_K1B_BLOCK=1024" \
  --variant=";CVD_NO_LDSF=1;CVD_K1B_BLOCK=512" --variant= --variant=";CVD_K1B_BLOCK=512;CVD_FILTER_MAX_LOG2=14" \
  --p 0.01 0.02 --rounds 3 --out $O/ab_block.jsonl > $O/ab_block.log 2>&1 || { echo "AB FAILED"; tail -20 $O/ab_block.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r03x2/ab_block.jsonl"):
    d = json.loads(l); print(d["p"], {k: round(v, 1) for k, v in d["median"].items()})
PY
