#!/bin/bash
# round 3 evidence, part 2: C4 on one GPU (the default 1e8 trials over N x p), then the
# m6 sweep rocprofv3 trace + PMC on the final tree
set -uo pipefail
O=gpurun_out/r03h
mkdir -p $O
timeout -k 10 900 python -u bench.py --config c4 > $O/bench_c4.json 2> $O/bench_c4.err \
  || { echo "C4 FAILED"; tail -20 $O/bench_c4.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c4.json').read().strip().splitlines()[-1]); print('c4', round(d['value']), 'trials/s total', {k: round(v['trials_per_s']) for k, v in d['per_N'].items()})"
bash profiles/collect_sweep.sh $O/m6 m6 || { echo "COLLECT FAILED"; exit 1; }
echo ALL DONE
