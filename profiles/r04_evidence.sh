#!/bin/bash
# Round 4 evidence at HEAD: rocprofv3 kernel trace + stats of each config's bench line and
# the per-p PMC passes (profiles/collect_sweep.sh), for profiles/summarize.py.
set -uo pipefail
OUT=$1; shift
for c in m6 m2 r23_m4; do
  timeout -k 10 900 bash profiles/collect_sweep.sh $OUT/$c $c > $OUT.$c.log 2>&1 || { echo "collect $c failed"; tail -20 $OUT.$c.log; exit 1; }
  echo "$c collected"
done
