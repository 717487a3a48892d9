#!/bin/bash
# Round 6: the lockstep launch's sensitivity to VALU issue -- CVD_K1S_PADV extra independent
# v_bitop3 per step (timing ablation, sums unchanged), same box, p = 0.05 and 0.2.
#   bash profiles/r06_padv.sh gpurun_out/r06w
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
for p in 0.05 0.2; do
  for k in 0 8 16 32 0; do
    run p${p}_pad${k}_$RANDOM CVD_JIT_DEFINES=-DCVD_K1S_PADV=$k -- --p $p --steps 2 --warmup 1
  done
done
