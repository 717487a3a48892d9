#!/bin/bash
# Round 4 (option since removed from bench.py): C3 with the H1 and H2 generator launches on two queues (--gen-queues 2)
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
summ() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],round(d['value']),'ms/step',round(d['ms_per_step'],2),'gen',round(d['diagnostic'].get('generator_ms_per_step',0),2),'det',round(d['diagnostic'].get('detector_ms_per_step',0),2),d['diagnostic']['per_p']==d['diagnostic']['per_p'])" $1; }
B="python bench.py --cpu-baseline 0 --early-decision 0 --config r23_m4"
for i in 1 2; do
  for q in 1 2; do
    timeout -k 10 300 $B --gen-queues $q > $OUT/bench_r23_q$q.$i.json 2> $OUT/bench_r23_q$q.$i.err || { tail -5 $OUT/bench_r23_q$q.$i.err; exit 1; }
    summ $OUT/bench_r23_q$q.$i.json
  done
done
python -c "
import json
a=json.loads(open('$OUT/bench_r23_q1.1.json').read().strip().splitlines()[-1]); b=json.loads(open('$OUT/bench_r23_q2.1.json').read().strip().splitlines()[-1])
print('per-p counts equal:', a['diagnostic']['per_p']==b['diagnostic']['per_p'])"
