#!/bin/bash
# Round 4: new GPU tests (grid ABI, fused slicing, walk flags), then the equal-weighted
# m6 sweep step with the detector launches on 1 / 3 device queues and 3 / 4 rounds per p.
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_grid.py tests/test_gpu_walk.py tests/test_gpu_fused.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
run() {  # name args...
  local nm=$1; shift
  timeout -k 10 400 python bench.py --config m6 --cpu-baseline 0 --early-decision 0 "$@" > $OUT/$nm.json 2> $OUT/$nm.err || { tail -5 $OUT/$nm.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/$nm.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$nm',round(d['value']),'ms/step',round(d['ms_per_step'],1),'phase',round(r['detector_phase_ms'],1),'launch',round(r['avg_launch_ms'],1),'gen',round(d['diagnostic']['generator_ms_per_step'],1),{k:round(v) for k,v in d['diagnostic']['detector_ms_by_p'].items()})"
}
run s3_b3 --steps 3 --warmup 1 --streams 3
run s1_b3 --steps 3 --warmup 1 --streams 1
run s2_b3 --steps 3 --warmup 1 --streams 2
run s3_b4 --steps 3 --warmup 1 --streams 3 --batch 524288
run s6_b3 --steps 3 --warmup 1 --streams 6
