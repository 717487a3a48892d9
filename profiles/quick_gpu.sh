#!/bin/bash
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for c in m6 m2 r23_m4; do
  timeout -k 10 600 python bench.py --config $c --cpu-baseline 0 --early-decision 0 > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 1
  python -c "import json;d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],'gen',d['diagnostic']['generator_ms_per_step'],'det',d['diagnostic']['detector_ms_per_step'])"
done
