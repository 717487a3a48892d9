#!/bin/bash
# Round 4: what the equal-weighted sweep step costs against single-p launches of 20
# residency rounds (round 3's step) on the same box, and the launch-size / queue options.
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name args...
  local nm=$1; shift
  timeout -k 10 400 python bench.py --config m6 --cpu-baseline 0 --early-decision 0 "$@" > $OUT/$nm.json 2> $OUT/$nm.err || { tail -5 $OUT/$nm.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/$nm.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$nm',round(d['value']),'ms/step',round(d['ms_per_step'],1),'det',round(r['detector_ms_per_step'],1),'gen',round(d['diagnostic']['generator_ms_per_step'],1),[(x['p'],round(x['ms'],1)) for x in d['diagnostic']['detector_ms_by_launch']])"
}
run multi_b3 --steps 3 --warmup 1
run multi_b3_q2 --steps 3 --warmup 1 --group-streams 2
run multi_b5 --steps 2 --warmup 1 --batch 655360
for p in 0.01 0.02 0.05 0.1 0.15 0.2; do
  run single20_$p --steps 1 --warmup 1 --batch 2621440 --p $p
done
