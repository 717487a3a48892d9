#!/bin/bash
# Round 4: C3 step size (--batch: trials per step) for the overlapped pipeline
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
summ() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],round(d['value']),'ms/step',round(d['ms_per_step'],2),'gen',round(d['diagnostic'].get('generator_ms_per_step',0),2),'det',round(d['diagnostic'].get('detector_ms_per_step',0),2))" $1; }
B="python bench.py --cpu-baseline 0 --early-decision 0 --config r23_m4"
for i in 1 2; do
  for b in ${BATCHES:-131072 262144 524288}; do
    timeout -k 10 300 $B --batch $b > $OUT/bench_r23_B$b.$i.json 2> $OUT/bench_r23_B$b.$i.err || { tail -5 $OUT/bench_r23_B$b.$i.err; exit 1; }
    summ $OUT/bench_r23_B$b.$i.json
  done
done
