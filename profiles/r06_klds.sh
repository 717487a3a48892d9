#!/bin/bash
# Round 6: the six flip / canonicalisation masks read from a block-shared LDS table instead of a
# v_mov per use group (CVD_BS_KLDS=1; 122 VGPRs, no scratch): the parity suites under it, then the
# six-p sweep, three alternating rounds on one box.
#   bash profiles/r06_klds.sh gpurun_out/r06ar
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
CVD_JIT_DEFINES=-DCVD_BS_KLDS=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walk.py \
  tests/test_gpu_multi.py tests/test_gpu_configs.py tests/test_gpu_early.py tests/test_gpu_chunked.py tests/test_gpu_c0.py \
  -x -q --timeout 240 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for rep in 1 2 3; do
  for e in 1 0; do
    CVD_JIT_DEFINES=-DCVD_BS_KLDS=$e timeout -k 10 300 python3 bench.py --cpu-baseline 0 --early-decision 0 --steps 6 --warmup 1 \
      > "$OUT/sweep_klds${e}_$rep.json" 2> "$OUT/sweep_klds${e}_$rep.err" || { tail -5 "$OUT/sweep_klds${e}_$rep.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/sweep_klds${e}_$rep.json').read().strip().splitlines()[-1]);print('klds=$e rep=$rep',round(d['value']),[round(x['ms']) for x in d['diagnostic']['detector_ms_by_launch']])"
  done
done
