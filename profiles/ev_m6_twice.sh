#!/bin/bash
# Parity tests of the detector paths, then two m6 headline bench runs (per-p detector ms).
set -uo pipefail
OUT=$1; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_jit_variants.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 --early-decision 0 > $OUT/m6_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('$OUT/m6_$i.json').read().strip().splitlines()[-1]);print(round(d['value']),{k:round(v) for k,v in d['diagnostic']['detector_ms_by_p'].items()})"
done
