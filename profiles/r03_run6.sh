#!/bin/bash
# round 3, GPU call 6: small-table LDS image (log T_ref per entry, next as entry base)
# for the table walks -- parity tests, C1/C3 bench lines fused and unfused
set -uo pipefail
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_configs.py tests/test_gpu_parity.py \
  tests/test_gpu_exponent.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for cfg in m2 r23_m4; do
  for f in 1 0; do
    timeout -k 10 300 python -u bench.py --config $cfg --fused $f --cpu-baseline 0 > $O/bench_${cfg}_fused$f.json 2> $O/bench_${cfg}_fused$f.err \
      || { echo "BENCH $cfg $f FAILED"; tail -20 $O/bench_${cfg}_fused$f.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${cfg}_fused$f.json').read().strip().splitlines()[-1]); print('$cfg fused=$f', round(d['value']/1e6,3), 'M trials/s', round(d['ms_per_step'],2), 'ms/step gen', round(d['diagnostic']['generator_ms_per_step'],2), 'det', round(d['diagnostic']['detector_ms_per_step'],2), 'early_eq', d.get('early_decision',{}).get('counts_equal_full_run'))"
  done
done
echo ALL DONE
