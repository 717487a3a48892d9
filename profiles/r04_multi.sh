#!/bin/bash
# Round 4: multi-model launches (cvd_detect_multi) -- tests, then the equal-weighted m6
# sweep step with one launch per p vs multi-model launches, at 3 and 4 rounds per p.
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_multi.py tests/test_gpu_grid.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
run() {  # name args...
  local nm=$1; shift
  timeout -k 10 400 python bench.py --config m6 --cpu-baseline 0 --early-decision 0 "$@" > $OUT/$nm.json 2> $OUT/$nm.err || { tail -5 $OUT/$nm.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/$nm.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$nm',round(d['value']),'ms/step',round(d['ms_per_step'],1),'det',round(r['detector_ms_per_step'],1),'gen',round(d['diagnostic']['generator_ms_per_step'],1),[(x['p'],round(x['ms'],1)) for x in d['diagnostic']['detector_ms_by_launch']])"
}
run multi_b3 --steps 3 --warmup 1
run single_b3 --steps 3 --warmup 1 --multi 0
run multi_b4 --steps 3 --warmup 1 --batch 524288
run multi_b336 --steps 3 --warmup 1 --batch 436906
