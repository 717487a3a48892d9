#!/bin/bash
# Round 4 (option since removed from bench.py): C3 with the overlapped generator stream at high HIP priority (--gen-priority -1)
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
summ() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],round(d['value']),'ms/step',round(d['ms_per_step'],2),'gen',round(d['diagnostic'].get('generator_ms_per_step',0),2),'det',round(d['diagnostic'].get('detector_ms_per_step',0),2))" $1; }
B="python bench.py --cpu-baseline 0 --early-decision 0 --config r23_m4"
for i in 1 2; do
  for pr in 0 -1; do
    timeout -k 10 300 $B --gen-priority $pr > $OUT/bench_r23_p$pr.$i.json 2> $OUT/bench_r23_p$pr.$i.err || { tail -5 $OUT/bench_r23_p$pr.$i.err; exit 1; }
    summ $OUT/bench_r23_p$pr.$i.json
  done
done
