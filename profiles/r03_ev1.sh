#!/bin/bash
# round 3 evidence, part 1: full GPU suite, smoke, the driver's bench command, and the
# default bench lines of the secondary configs with their CPU baselines
set -uo pipefail
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 \
  || { echo "GPU TESTS FAILED"; tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err \
  || { echo "BENCH FAILED"; tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print('m6', round(d['value']), 'trials/s', round(d['ms_per_step'],1), 'ms/step', 'traffic x', round(d['roofline']['traffic_x_algorithmic'] or -1,2), 'cpu', round(d['cpu_baseline']['value'],1), 'pd_match', d['pd_match_vs_cpu']['match'], 'c0', d['c0_demo']['match'])"
for cfg in m2 r23_m4; do
  timeout -k 10 400 python -u bench.py --config $cfg > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { echo "BENCH $cfg FAILED"; tail -20 $O/bench_$cfg.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$cfg.json').read().strip().splitlines()[-1]); print('$cfg', round(d['value']/1e6,3), 'M trials/s', 'cpu', round(d['cpu_baseline']['value'],1), 'pd_match', d['pd_match_vs_cpu']['match'])"
done
echo ALL DONE
