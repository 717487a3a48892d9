#!/bin/bash
# round 3, GPU call 4: fused trial kernel (generator + LDS table automaton) and device
# rows ordered by visits -- parity tests, A/B of the row order, C1/C3 bench lines fused
# and unfused
set -uo pipefail
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_configs.py \
  tests/test_gpu_bfs.py tests/test_gpu_learn.py tests/test_gpu_early.py tests/test_gpu_cli.py \
  -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u profiles/ab_k1b.py --variant= "--variant=;CVD_ROW_ORDER=first" --p 0.01 0.02 0.05 0.1 0.2 \
  --rounds 3 --out $O/ab_roworder.jsonl > $O/ab.log 2>&1 || { echo "AB FAILED"; tail -20 $O/ab.log; exit 1; }
grep median $O/ab.log | python3 -c "import sys,json; [print(json.loads(l)['p'], json.loads(l)['median']) for l in sys.stdin]"
for cfg in m2 r23_m4; do
  for f in 1 0; do
    timeout -k 10 300 python -u bench.py --config $cfg --fused $f --cpu-baseline 0 > $O/bench_${cfg}_fused$f.json 2> $O/bench_${cfg}_fused$f.err \
      || { echo "BENCH $cfg $f FAILED"; tail -20 $O/bench_${cfg}_fused$f.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${cfg}_fused$f.json').read().strip().splitlines()[-1]); print('$cfg fused=$f', round(d['value']/1e6,3), 'M trials/s', round(d['ms_per_step'],2), 'ms/step gen', round(d['diagnostic']['generator_ms_per_step'],2), 'det', round(d['diagnostic']['detector_ms_per_step'],2), 'early_eq', d.get('early_decision',{}).get('counts_equal_full_run'))"
  done
done
echo ALL DONE
