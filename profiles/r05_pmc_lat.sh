#!/bin/bash
# Memory-latency counters of the m = 6 detector at one p (run on the GPU box from the repo
# root):  bash profiles/r05_pmc_lat.sh OUTDIR P
# rocprofv3 -L first (the counter list of this box), then one --pmc pass per group over one
# bench launch at p (--steps 1 --warmup 0), each under its own time limit.
set -uo pipefail
OUT=${1:?out dir}; P=${2:-0.05}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
ARGS="--config m6 --cpu-baseline 0 --early-decision 0 --p $P --steps 1 --warmup 0"
i=0
for grp in "SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU" \
           "TCC_HIT_sum TCC_MISS_sum" \
           "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp -T --output-format csv -d "$ROOT/$OUT/pmc$i" -o run \
    -- python3 bench.py $ARGS > "$OUT/bench_pmc$i.json" 2> "$OUT/pmc$i.err" || echo "pass $i ($grp) failed rc=$?" >&2
  echo "pass $i ($grp) done" >&2
done
