#!/bin/bash
# Round 6: walk-mode record forms at p = 0.01 / 0.02 (one box): the two-step 32-B records (default)
# against the single-step 16-B dense records (CVD_WALK_NOT2=1: drow, 64 B per row), whole launches
# and H1 waves alone (-DCVD_WALK_ABL=4, timing only), and bursts of 8 / 16 single steps.
#   bash profiles/r06_walkrec.sh gpurun_out/r06r
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
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
  run p01_t2_$rep X=1 -- --p 0.01 --steps 3 --warmup 1
  run p01_not2_$rep CVD_WALK_NOT2=1 -- --p 0.01 --steps 3 --warmup 1
done
run p01_not2_b8 CVD_WALK_NOT2=1 CVD_WALK_BURST=8 -- --p 0.01 --steps 3 --warmup 1
run p01_t2_h1 CVD_JIT_DEFINES=-DCVD_WALK_ABL=4 -- --p 0.01 --steps 2 --warmup 1
run p01_not2_h1 CVD_WALK_NOT2=1 CVD_JIT_DEFINES=-DCVD_WALK_ABL=4 -- --p 0.01 --steps 2 --warmup 1
run p01_t2c_h1 CVD_WALK_T2C=1 CVD_JIT_DEFINES=-DCVD_WALK_ABL=4 -- --p 0.01 --steps 2 --warmup 1
run p02_walk_not2 CVD_WALK=1 CVD_WALK_NOT2=1 -- --p 0.02 --steps 3 --warmup 1
run p02_walk_t2 CVD_WALK=1 -- --p 0.02 --steps 3 --warmup 1
run p02_lock CVD_WALK=0 -- --p 0.02 --steps 3 --warmup 1
