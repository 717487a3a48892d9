#!/bin/bash
# Round 4: grid/multi/run_experiment tests, then the bench line in both sweep modes
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_grid.py tests/test_gpu_multi.py tests/test_gpu_distributed.py tests/test_gpu_cli.py tests/test_gpu_configs.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
run() {  # name args...
  local nm=$1; shift
  timeout -k 10 500 python bench.py --cpu-baseline 0 "$@" > $OUT/$nm.json 2> $OUT/$nm.err || { tail -5 $OUT/$nm.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/$nm.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$nm',round(d['value']),'wall',round(d['value_wall']),'ms/step',round(d['ms_per_step'],1),'det',round(r['detector_ms_per_step'],1),'gen',round(d['diagnostic']['generator_ms_per_step'],1),[(x['p'],round(x['ms'],1)) for x in d['diagnostic']['detector_ms_by_launch']], 'early', d.get('early_decision',{}).get('counts_equal_full_run'))"
}
run perp6 --config m6 --steps 6 --warmup 1
run perp8 --config m6 --steps 8 --warmup 1 --early-decision 0
run all2 --config m6 --steps 2 --warmup 1 --sweep all --early-decision 0
run m2 --config m2 --early-decision 0
run r23 --config r23_m4 --early-decision 0
