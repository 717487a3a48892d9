#!/bin/bash
# Round 4: the stride-3 rate-2/3 encoder -- generator/stream parity tests, then the C3 line
# and a generator PMC pass
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_configs.py tests/test_gpu_grid.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python bench.py --config r23_m4 --cpu-baseline 0 --early-decision 0 > $OUT/bench_r23.json 2> $OUT/bench_r23.err || { tail -5 $OUT/bench_r23.err; exit 1; }
python -c "import json;d=json.loads(open('$OUT/bench_r23.json').read().strip().splitlines()[-1]);print('r23',round(d['value']),'ms/step',round(d['ms_per_step'],2),'gen',round(d['diagnostic']['generator_ms_per_step'],2),'det',round(d['diagnostic']['detector_ms_per_step'],2))"
timeout -k 10 300 python bench.py --config r23_m4 --cpu-baseline 0 --early-decision 0 --overlap 0 > $OUT/bench_r23_noov.json 2> $OUT/bench_r23_noov.err || { tail -5 $OUT/bench_r23_noov.err; exit 1; }
python -c "import json;d=json.loads(open('$OUT/bench_r23_noov.json').read().strip().splitlines()[-1]);print('r23 no-overlap',round(d['value']),'ms/step',round(d['ms_per_step'],2),'gen',round(d['diagnostic']['generator_ms_per_step'],2),'det',round(d['diagnostic']['detector_ms_per_step'],2))"
