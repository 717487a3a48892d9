#!/bin/bash
# Round 6: a focused GPU suite and the headline twice (the default tree).
#   bash profiles/r06_verify.sh gpurun_out/r06l [pytest files...]
set -uo pipefail
OUT=${1:?out dir}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -x -q --timeout 240 --timeout-method thread > "$OUT/tests.log" 2>&1 \
    || { tail -20 "$OUT/tests.log"; exit 1; }
  tail -1 "$OUT/tests.log"
fi
B="--cpu-baseline 0 --early-decision 0 --steps 6 --warmup 1"
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py $B > "$OUT/hl_$rep.json" 2> "$OUT/hl_$rep.err" || { tail -5 "$OUT/hl_$rep.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/hl_$rep.json').read().strip().splitlines()[-1]);print('headline',round(d['value']),[round(x['ms'],1) for x in d['diagnostic']['detector_ms_by_launch']])"
done
