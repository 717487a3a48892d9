#!/bin/bash
# Round 6: the two-step lookup pipeline of the lockstep loop (CVD_K1S_DEEP=1; =2 the hash before the wait) against the
# one-step cursor (=0): the parity suites, then same-box launches at the lockstep p.
#   bash profiles/r06_deep.sh gpurun_out/r06u
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walk.py tests/test_gpu_multi.py \
  tests/test_gpu_configs.py tests/test_gpu_early.py tests/test_gpu_chunked.py tests/test_gpu_c0.py -x -q \
  --timeout 240 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
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
  for d in 2 1 0; do
    for p in 0.05 0.1 0.2; do
      run p${p}_deep${d}_$rep CVD_JIT_DEFINES=-DCVD_K1S_DEEP=$d -- --p $p --steps 2 --warmup 1
    done
  done
done
