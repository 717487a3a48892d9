#!/bin/bash
# Round 4 (options since removed from bench.py): m6 with the generator overlapped at a lower dispatch priority than the detector
# (--overlap 1 --det-priority -1: the generator only takes CU slots the detector's pending
# blocks do not claim, i.e. its launch tails), at a batch whose two buffers fit
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
summ() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],round(d['value']),'ms/step',round(d['ms_per_step'],2),'gen',round(d['diagnostic'].get('generator_ms_per_step',0),2),'det',round(d['diagnostic'].get('detector_ms_per_step',0),2))" $1; }
B="python bench.py --cpu-baseline 0 --early-decision 0 --config m6 --batch ${BATCH:-655360} --steps 6 --warmup 1"
for i in 1 2; do
  for v in ov0 ov1 ov1d ov1g; do
    case $v in ov0) A="--overlap 0";; ov1) A="--overlap 1";; ov1d) A="--overlap 1 --det-priority -1";; ov1g) A="--overlap 1 --gen-priority -1";; esac
    timeout -k 10 300 $B $A > $OUT/bench_m6_$v.$i.json 2> $OUT/bench_m6_$v.$i.err || { tail -5 $OUT/bench_m6_$v.$i.err; exit 1; }
    summ $OUT/bench_m6_$v.$i.json
  done
done
