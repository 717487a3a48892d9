#!/bin/bash
# Round 6: lockstep units alternating H1 / H2 waves (-DCVD_K1S_MIX=1) against units in order.
#   bash profiles/r06_mix.sh gpurun_out/r06k
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
CVD_JIT_DEFINES=-DCVD_K1S_MIX=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walk.py \
  tests/test_gpu_multi.py -x -q --timeout 240 --timeout-method thread > "$OUT/tests_mix.log" 2>&1 \
  || { tail -20 "$OUT/tests_mix.log"; exit 1; }
tail -1 "$OUT/tests_mix.log"
B="--cpu-baseline 0 --early-decision 0 --steps 6 --warmup 1"
for rep in 1 2; do for mx in 0 1; do
  CVD_JIT_DEFINES=-DCVD_K1S_MIX=$mx timeout -k 10 300 python3 bench.py $B > "$OUT/hl_mix${mx}_$rep.json" 2> "$OUT/hl_mix${mx}_$rep.err" || { tail -5 "$OUT/hl_mix${mx}_$rep.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/hl_mix${mx}_$rep.json').read().strip().splitlines()[-1]);print('mix=$mx',round(d['value']),[round(x['ms'],1) for x in d['diagnostic']['detector_ms_by_launch']])"
done; done
