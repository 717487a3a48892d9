#!/bin/bash
# Round 6: where the candidate test and its directory loads sit in the step (CVD_K1S_MIDPOS:
# 0 between the words' ACS, 1 at the step start, 2 after the ACS); ordering only, same sums.
#   bash profiles/r06_midpos.sh gpurun_out/r06o
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
CVD_JIT_DEFINES=-DCVD_K1S_MIDPOS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 \
  --timeout-method thread -k "m6" > "$OUT/tests_mid1.log" 2>&1 || { tail -20 "$OUT/tests_mid1.log"; exit 1; }
tail -1 "$OUT/tests_mid1.log"
B="--cpu-baseline 0 --early-decision 0 --steps 6 --warmup 1"
for rep in 1 2; do for mp in 0 1 2; do
  CVD_JIT_DEFINES=-DCVD_K1S_MIDPOS=$mp timeout -k 10 150 python3 bench.py $B > "$OUT/hl_mid${mp}_$rep.json" 2> "$OUT/hl_mid${mp}_$rep.err" || { tail -5 "$OUT/hl_mid${mp}_$rep.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/hl_mid${mp}_$rep.json').read().strip().splitlines()[-1]);print('midpos=$mp',round(d['value']),[round(x['ms'],1) for x in d['diagnostic']['detector_ms_by_launch']])"
done; done
