#!/bin/bash
# Collect the rocprofv3 evidence committed under profiles/ (run on the GPU box,
# from the repo root, e.g. via gpurun).  Kernel trace/stats and each PMC group
# run in separate passes (no --pmc together with sys/runtime traces).
#   bash profiles/collect.sh gpurun_out/prof "--cpu-baseline 0"
set -euo pipefail
OUT=${1:-gpurun_out/prof}
ARGS=${2:-"--cpu-baseline 0 --early-decision 0"}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$ROOT/$OUT/trace" -o run \
  -- python3 bench.py $ARGS > "$OUT/bench_trace.json"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $grp -T --output-format csv -d "$ROOT/$OUT/pmc$i" -o run \
    -- python3 bench.py $ARGS --steps 2 --warmup 0 > "$OUT/bench_pmc$i.json"
done
echo "profiles collected in $OUT"
