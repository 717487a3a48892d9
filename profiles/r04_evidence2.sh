#!/bin/bash
# Round 4 final evidence at HEAD, part 2: rocprofv3 kernel trace + stats and the per-p
# PMC passes (profiles/collect_sweep.sh) of the m6 and r23 bench lines
set -uo pipefail
OUT=$1; shift
for c in m6 r23_m4; do
  timeout -k 10 900 bash profiles/collect_sweep.sh $OUT/$c $c > $OUT.$c.log 2>&1 || { echo "collect $c failed"; tail -20 $OUT.$c.log; exit 1; }
  echo "$c collected"
done
