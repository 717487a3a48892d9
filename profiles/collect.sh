#!/bin/bash
# Collect the rocprofv3 evidence committed under profiles/ (run on the GPU box,
# from the repo root, e.g. via gpurun).  Kernel trace/stats and each PMC group
# run in separate passes (no --pmc together with sys/runtime traces).
set -euo pipefail
OUT=${1:-gpurun_out/prof}
ARGS=${2:-"--cpu-baseline 0"}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$ROOT/$OUT/trace" -o run \
  -- python3 bench.py $ARGS > "$OUT/bench_trace.json"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$ROOT/$OUT/pmc_fetch" -o run \
  -- python3 bench.py $ARGS --steps 2 --warmup 0 > "$OUT/bench_pmc_fetch.json"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$ROOT/$OUT/pmc_write" -o run \
  -- python3 bench.py $ARGS --steps 2 --warmup 0 > "$OUT/bench_pmc_write.json"
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T \
  --output-format csv -d "$ROOT/$OUT/pmc_sq" -o run \
  -- python3 bench.py $ARGS --steps 2 --warmup 0 > "$OUT/bench_pmc_sq.json"
echo "profiles collected in $OUT"
