#!/bin/bash
# round 3: LDS-resident Bloom filter for walking models (CVD_K1B_LDSF, 1,024-thread blocks,
# filter <= 128 KiB) and 1,024 filter patterns: parity tests, then A/B against the
# global-memory filter (CVD_NO_LDSF=1)
set -uo pipefail
O=gpurun_out/r03x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 240 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 500 python -u profiles/ab_k1b.py --variant= --variant=";CVD_NO_LDSF=1" --p 0.01 0.02 0.1 0.2 \
  --rounds 3 --out $O/ab_ldsf.jsonl > $O/ab_ldsf.log 2>&1 || { echo "AB FAILED"; tail -20 $O/ab_ldsf.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r03x/ab_ldsf.jsonl"):
    d = json.loads(l); print(d["p"], {k: round(v, 1) for k, v in d["median"].items()})
PY
