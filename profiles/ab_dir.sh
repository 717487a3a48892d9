#!/bin/bash
# Directory load factor and filter-positive load placement under the interleaved
# slots: one bench.py --p launch per (variant, p), m6 headline batch.
set -uo pipefail
OUT=${1:-gpurun_out/r02z6_dir}; mkdir -p $OUT; export TMPDIR=/tmp
run() {  # name env...
  local name=$1; shift
  for p in 0.1 0.01; do
    env "$@" timeout -k 10 300 python bench.py --cpu-baseline 0 --early-decision 0 --p $p --steps 3 --warmup 1 > $OUT/$name.p$p.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads(open('$OUT/$name.p$p.json').read().strip().splitlines()[-1]);print('$name','p=$p',round(d['diagnostic']['detector_ms_per_step'],1))"
  done
}
run base CVD_NOP=1
run load4 CVD_DIR_LOAD_LOG2=2
run load16 CVD_DIR_LOAD_LOG2=4
run mid1 CVD_JIT_DEFINES=-DCVD_K1B_MID=1
run mid3 CVD_JIT_DEFINES=-DCVD_K1B_MID=3
run base2 CVD_NOP=1
