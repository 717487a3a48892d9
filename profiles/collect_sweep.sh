#!/bin/bash
# rocprofv3 evidence for one bench config over its WHOLE p sweep (run on the GPU box
# from the repo root, e.g. via gpurun):
#   bash profiles/collect_sweep.sh gpurun_out/r03_m6 m6
# One --kernel-trace --stats pass of the default bench line (the judged command), then
# one --pmc pass per counter group (never combined with a trace domain), each over one
# launch per p of the sweep (--steps = number of p, --warmup 0: step s runs p_grid[s]),
# so that profiles/summarize.py can give per-p rows and the launch-weighted sweep mean.
set -euo pipefail
OUT=${1:?out dir}
CFG=${2:-m6}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
case "$CFG" in
  m2) STEPS=1 ;;
  *) STEPS=6 ;;
esac
ARGS="--config $CFG --cpu-baseline 0 --early-decision 0 ${EXTRA_ARGS:-}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$ROOT/$OUT/trace" -o run \
  -- python3 bench.py $ARGS > "$OUT/bench_trace.json"
i=0
for grp in "FETCH_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $grp -T --output-format csv -d "$ROOT/$OUT/pmc$i" -o run \
    -- python3 bench.py $ARGS --steps $STEPS --warmup 0 > "$OUT/bench_pmc$i.json"
  echo "pass $i ($grp) done" >&2
done
echo "profiles collected in $OUT"
