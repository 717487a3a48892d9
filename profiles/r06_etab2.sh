#!/bin/bash
# Round 6: the ACS's mu-specific addend planes from an LDS table (CVD_BS_ETAB2=1: 8 VALU fewer per
# step, static loop cost 3,260 -> 3,168 cycles per six steps): the parity suites under it, then
# same-box launches at every p, two rounds.
#   bash profiles/r06_etab2.sh gpurun_out/r06aa
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
CVD_JIT_DEFINES=-DCVD_BS_ETAB2=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walk.py \
  tests/test_gpu_multi.py tests/test_gpu_configs.py tests/test_gpu_early.py tests/test_gpu_chunked.py tests/test_gpu_c0.py \
  -x -q --timeout 240 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
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
  for p in 0.01 0.02 0.05 0.1 0.15 0.2; do
    run p${p}_etab1_$rep CVD_JIT_DEFINES=-DCVD_BS_ETAB2=1 -- --p $p --steps 2 --warmup 1
    run p${p}_etab0_$rep CVD_JIT_DEFINES=-DCVD_BS_ETAB2=0 -- --p $p --steps 2 --warmup 1
  done
done
