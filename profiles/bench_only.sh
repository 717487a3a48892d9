#!/bin/bash
# Headline + C1 + C3 bench lines only (no tests): quick A/B of a kernel change.
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
for c in m6 m2 r23_m4; do
  timeout -k 10 600 python bench.py --config $c --cpu-baseline 0 --early-decision 0 "$@" > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 1
  python -c "import json;d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],'gen',d['diagnostic']['generator_ms_per_step'],'det',d['diagnostic']['detector_ms_per_step'])"
done
