#!/bin/bash
# Round 6: p = 0.05 (315,953 rows) with the whole filter in LDS (CVD_LDSF_MAX_ROWS=400000) against
# the default pre-filter + L2 filter, two alternating rounds on one box.
#   bash profiles/r06_p02ldsf.sh gpurun_out/r06al
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for m in pf ldsf; do
    case $m in pf) E="X=1";; ldsf) E="CVD_LDSF_MAX_ROWS=400000";; esac
    env $E timeout -k 10 180 python3 bench.py --cpu-baseline 0 --early-decision 0 --p 0.05 --steps 3 --warmup 1 \
      > "$OUT/p05_${m}_$rep.json" 2> "$OUT/p05_${m}_$rep.err" || { tail -5 "$OUT/p05_${m}_$rep.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/p05_${m}_$rep.json').read().strip().splitlines()[-1]);print('p=0.05 $m',round(d['roofline']['avg_launch_ms'],1),d['diagnostic']['lds_filter_by_p'])"
  done
done
