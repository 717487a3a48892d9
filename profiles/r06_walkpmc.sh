#!/bin/bash
# Round 6: L2 hit rate and latency of the walk launch (p = 0.01) with the two-step records
# (default) and the single-step dense records (CVD_WALK_NOT2=1); one --pmc pass per run.
#   bash profiles/r06_walkpmc.sh gpurun_out/r06s
set -uo pipefail
OUT=${1:?out dir}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--cpu-baseline 0 --early-decision 0 --p 0.01 --steps 1 --warmup 0"
for form in t2 not2; do
  if [ $form = not2 ]; then export CVD_WALK_NOT2=1; else unset CVD_WALK_NOT2; fi
  i=0
  for grp in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" "VmemLatency" "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAVES"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $grp -T --output-format csv -d "$ROOT/$OUT/${form}_pmc$i" -o run \
      -- python3 bench.py $ARGS > "$OUT/${form}_pmc$i.json" 2> "$OUT/${form}_pmc$i.err" || { echo "pass $form $i failed"; exit 1; }
    echo "pass $form $i ($grp) done"
  done
done
