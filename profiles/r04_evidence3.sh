#!/bin/bash
# Round 4 final evidence at HEAD, part 2: rocprofv3 kernel trace + stats and the per-p
# PMC passes of the m6 and r23 bench lines (profiles/collect_sweep.sh), then C4
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
for c in m6 r23_m4; do
  timeout -k 10 900 bash profiles/collect_sweep.sh $OUT/$c $c > $OUT/collect_$c.log 2>&1 || { echo "collect $c failed"; tail -20 $OUT/collect_$c.log; exit 1; }
  echo "$c collected"
done
timeout -k 10 900 python -u bench.py --config c4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -5 $OUT/bench_c4.err; exit 1; }
python -c "import json;d=json.loads(open('$OUT/bench_c4.json').read().strip().splitlines()[-1]);print('c4',round(d['value']),{k:round(v['trials_per_s']) for k,v in d['per_N'].items()})"
