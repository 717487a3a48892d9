#!/bin/bash
# Memory-pipeline counters of the m = 6 detector at one p (GPU box, repo root):
#   bash profiles/r05_pmc_mem.sh OUTDIR P
# derived rocprofv3 metrics, one per pass: VmemLatency (cycles per VMEM instruction),
# TA / TCC busy, MemUnitStalled (TCP data stalls, % of GPU time), LdsLatency
set -uo pipefail
OUT=${1:?out dir}; P=${2:-0.05}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--config m6 --cpu-baseline 0 --early-decision 0 --p $P --steps 1 --warmup 0"
i=0
for grp in "VmemLatency" "TA_BUSY_avr TCC_BUSY_avr GRBM_GUI_ACTIVE" "MemUnitStalled" "LdsLatency"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp -T --output-format csv -d "$ROOT/$OUT/pmc$i" -o run \
    -- python3 bench.py $ARGS > "$OUT/bench_pmc$i.json" 2> "$OUT/pmc$i.err" || echo "pass $i ($grp) failed rc=$?" >&2
  echo "pass $i ($grp) done" >&2
done
