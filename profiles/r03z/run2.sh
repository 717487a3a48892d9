#!/bin/bash
# round 3: the LDS-filter kernel with its own 1,024-pattern filter copy, the global filter
# back at 4,096 patterns: walk/parity tests, then A/B (full launch size)
set -uo pipefail
O=gpurun_out/r03z2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_parity.py tests/test_gpu_jit_variants.py -x -v --timeout 240 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u profiles/ab_k1b.py --trials 2621440 --variant= --variant=";CVD_NO_LDSF=1" --p 0.01 0.1 \
  --rounds 2 --out $O/ab_ldsf2.jsonl > $O/ab_ldsf2.log 2>&1 || { echo "AB FAILED"; tail -20 $O/ab_ldsf2.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r03z2/ab_ldsf2.jsonl"):
    d = json.loads(l); print(d["p"], {k: round(v, 1) for k, v in d["median"].items()})
PY
