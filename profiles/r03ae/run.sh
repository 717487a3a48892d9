#!/bin/bash
# round 3: generator noise exchange over 8 words per pass (default) against 4
# (CVD_GEN_CHUNK_WORDS=4): stream parity tests, then the m6 / r23 bench lines both ways
set -uo pipefail
O=gpurun_out/r03ae
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fused.py -x -q --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cw in 8 4; do
  for cfg in m6 r23_m4; do
    CVD_GEN_CHUNK_WORDS=$cw timeout -k 10 400 python -u bench.py --config $cfg --cpu-baseline 0 --early-decision 0 \
      > $O/bench_${cfg}_g$cw.json 2> $O/bench_${cfg}_g$cw.err || { echo "BENCH FAILED $cfg $cw"; tail -20 $O/bench_${cfg}_g$cw.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${cfg}_g$cw.json').read().strip().splitlines()[-1]); dg=d['diagnostic']; print('$cfg g$cw', round(d['value']), 'gen', round(dg['generator_ms_per_step'],2), 'det', round(dg['detector_ms_per_step'],2), 'step', round(d['ms_per_step'],2))"
  done
done
