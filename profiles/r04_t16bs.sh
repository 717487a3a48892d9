#!/bin/bash
# Round 4: C3 with the rate-2/3 detector in 512-thread blocks (CVD_T16_BIG_BLOCK=512)
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
summ() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],round(d['value']),'ms/step',round(d['ms_per_step'],2),'gen',round(d['diagnostic'].get('generator_ms_per_step',0),2),'det',round(d['diagnostic'].get('detector_ms_per_step',0),2))" $1; }
B="python bench.py --cpu-baseline 0 --early-decision 0 --config r23_m4"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_configs.py > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
CVD_T16_BIG_BLOCK=512 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_configs.py > $OUT/tests512.log 2>&1 || { tail -20 $OUT/tests512.log; exit 1; }
tail -n 1 $OUT/tests.log $OUT/tests512.log
for i in 1 2; do
  for v in 1024 512; do
    E="CVD_NOP=1"; [ $v = 512 ] && E="CVD_T16_BIG_BLOCK=512"
    env $E timeout -k 10 300 $B > $OUT/bench_r23_b$v.$i.json 2> $OUT/bench_r23_b$v.$i.err || { tail -5 $OUT/bench_r23_b$v.$i.err; exit 1; }
    summ $OUT/bench_r23_b$v.$i.json
    env $E timeout -k 10 300 $B --overlap 0 --steps 3 > $OUT/bench_r23_noov_b$v.$i.json 2> $OUT/bench_r23_noov_b$v.$i.err || { tail -5 $OUT/bench_r23_noov_b$v.$i.err; exit 1; }
    summ $OUT/bench_r23_noov_b$v.$i.json
  done
done
