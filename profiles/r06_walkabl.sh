#!/bin/bash
# Round 6: what the walk launch (p = 0.01) spends where (timing ablations, results differ):
# full, H1 waves only (-DCVD_WALK_ABL=4), H1 waves without their leavers' ACS steps (=12),
# H2 waves only (=1).
#   bash profiles/r06_walkabl.sh gpurun_out/r06n
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="--cpu-baseline 0 --early-decision 0 --p 0.01 --steps 3 --warmup 1"
for v in 12 8; do
  CVD_JIT_DEFINES=-DCVD_WALK_ABL=$v timeout -k 10 150 python3 bench.py $B > "$OUT/abl$v.json" 2> "$OUT/abl$v.err" || { tail -5 "$OUT/abl$v.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/abl$v.json').read().strip().splitlines()[-1]);print('abl=$v',round(d['roofline']['avg_launch_ms'],1))"
done
