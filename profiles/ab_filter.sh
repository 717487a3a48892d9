#!/bin/bash
# Filter size cap and the hash-only floor (CVD_ABL=32: hash + filter test, no key or
# record reads; wrong sums, timing only) under the interleaved 1/16 directory.
set -uo pipefail
OUT=${1:-gpurun_out/r02z8_filt}; mkdir -p $OUT; export TMPDIR=/tmp
run() {  # name env...
  local name=$1; shift
  for p in ${PS:-0.1 0.2 0.01}; do
    env "$@" timeout -k 10 300 python bench.py --cpu-baseline 0 --early-decision 0 --p $p --steps 3 --warmup 1 > $OUT/$name.p$p.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads(open('$OUT/$name.p$p.json').read().strip().splitlines()[-1]);print('$name','p=$p',round(d['diagnostic']['detector_ms_per_step'],1))"
  done
}
run base CVD_NOP=1
run filt4m CVD_FILTER_MAX_LOG2=20
run filt1m CVD_FILTER_MAX_LOG2=18


