#!/bin/bash
# the round-4 library (commit 0f984d0, built into ab_r04/, not tracked)
# against HEAD on ONE box, for C3 (--config r23_m4) and C1 (--config m2), alternating.
#   bash profiles/r06_ab_r04.sh gpurun_out/r06e
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="--cpu-baseline 0 --early-decision 0"
one() { # tree name args
  (cd "$1" && timeout -k 10 300 python3 bench.py $B $3) > "$OUT/$2.json" 2> "$OUT/$2.err" || { tail -5 "$OUT/$2.err"; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('$OUT/$2.json').read().strip().splitlines()[-1]);print('$2',round(d['value']),round(d['roofline']['avg_launch_ms'],2))"
}
for rep in 1 2; do
  one ab_r04 r04_c3_$rep "--config r23_m4 --steps 20 --warmup 5"
  one . head_c3_$rep "--config r23_m4 --steps 20 --warmup 5"
  one ab_r04 r04_c1_$rep "--config m2 --steps 6 --warmup 2"
  one . head_c1_$rep "--config m2 --steps 6 --warmup 2"
done
