#!/bin/bash
# Round 6: p = 0.01 walk mode (the default there) against lockstep (CVD_WALK=0) after the
# table-form ACS and mask-form cursor, two alternating rounds on one box.
#   bash profiles/r06_walk01.sh gpurun_out/r06ag
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for w in 1 0; do
    CVD_WALK=$w timeout -k 10 180 python3 bench.py --cpu-baseline 0 --early-decision 0 --p 0.01 --steps 3 --warmup 1 \
      > "$OUT/p01_walk${w}_$rep.json" 2> "$OUT/p01_walk${w}_$rep.err" || { tail -5 "$OUT/p01_walk${w}_$rep.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/p01_walk${w}_$rep.json').read().strip().splitlines()[-1]);print('p=0.01 walk=$w',round(d['roofline']['avg_launch_ms'],1))"
  done
done
