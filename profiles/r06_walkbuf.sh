#!/bin/bash
# Round 6: walk mode's stream as whole 16-B chunks refilled in wave-wide batches (CVD_WALK_BUF=1,
# 2) against one 4-B word load per word (=0): the walk suite, p = 0.01 launches, p = 0.02 and
# p = 0.05 with walk mode forced (CVD_WALK=1), and the lockstep p = 0.05 / 0.1 (whose variant
# compiles the same walk code).
#   bash profiles/r06_walkbuf.sh gpurun_out/r06q
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py -x -q --timeout 240 --timeout-method thread \
  > "$OUT/tests_walk.log" 2>&1 || { tail -20 "$OUT/tests_walk.log"; exit 1; }
tail -1 "$OUT/tests_walk.log"
run() {   # name, env..., then bench args after --
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 180 python3 bench.py --cpu-baseline 0 --early-decision 0 "$@" \
    > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -5 "$OUT/$name.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]);print('$name',round(d['roofline']['avg_launch_ms'],1))"
}
for rep in 1 2; do
  for b in 1 0 2; do
    run p01_buf${b}_$rep CVD_JIT_DEFINES=-DCVD_WALK_BUF=$b -- --p 0.01 --steps 3 --warmup 1
  done
done
run p01_buf1_h1only CVD_JIT_DEFINES="-DCVD_WALK_BUF=1 -DCVD_WALK_ABL=4" -- --p 0.01 --steps 2 --warmup 1
for b in 1 0; do
  run p02_walk_buf$b CVD_WALK=1 CVD_JIT_DEFINES=-DCVD_WALK_BUF=$b -- --p 0.02 --steps 3 --warmup 1
done
run p02_lock CVD_WALK=0 -- --p 0.02 --steps 3 --warmup 1
run p05_walk_buf1 CVD_WALK=1 CVD_JIT_DEFINES=-DCVD_WALK_BUF=1 -- --p 0.05 --steps 2 --warmup 1
for b in 1 0; do
  run p05_lock_buf$b CVD_JIT_DEFINES=-DCVD_WALK_BUF=$b -- --p 0.05 --steps 3 --warmup 1
  run p10_lock_buf$b CVD_JIT_DEFINES=-DCVD_WALK_BUF=$b -- --p 0.1 --steps 3 --warmup 1
done
