#!/bin/bash
# Round 6: the lookup's directory / filter masks in VGPRs (CVD_K1S_VMASK=1) and the filter load in
# the SGPR-base form (CVD_K1S_TRIM=2): static loop cost 3,260 -> 3,239 / 3,214 cycles per six
# steps; same-box launches at p = 0.05 and 0.15, two rounds.
#   bash profiles/r06_vmask.sh gpurun_out/r06y
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
  for p in 0.05 0.15; do
    run p${p}_base_$rep CVD_JIT_DEFINES=-DCVD_K1S_VMASK=0 -- --p $p --steps 2 --warmup 1
    run p${p}_vmask_$rep CVD_JIT_DEFINES=-DCVD_K1S_VMASK=1 -- --p $p --steps 2 --warmup 1
    run p${p}_vmtrim_$rep CVD_JIT_DEFINES="-DCVD_K1S_VMASK=1 -DCVD_K1S_TRIM=2" -- --p $p --steps 2 --warmup 1
  done
done
