#!/bin/bash
# Round 4: m6 step size -- 20 residency rounds (2,621,440 trials, default) against 30 (3,932,160)
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
summ() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],round(d['value']),'ms/step',round(d['ms_per_step'],2),[round(x['ms']) for x in d['diagnostic']['detector_ms_by_launch']])" $1; }
B="python bench.py --cpu-baseline 0 --early-decision 0 --config m6 --steps 6 --warmup 1"
for b in 2621440 3932160; do
  timeout -k 10 600 $B --batch $b > $OUT/bench_m6_B$b.json 2> $OUT/bench_m6_B$b.err || { tail -5 $OUT/bench_m6_B$b.err; exit 1; }
  summ $OUT/bench_m6_B$b.json
done
