#!/bin/bash
# Round 6: the table-form ACS (CVD_BS_ETAB2=1), with the next step's e0 read a step ahead (=2),
# against the select form (=0): the walk and parity suites under =2, then the six-p sweep
# (bench.py's default 6 steps, one per p), three alternating rounds on one box.
#   bash profiles/r06_etab2b.sh gpurun_out/r06ab
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
CVD_JIT_DEFINES=-DCVD_BS_ETAB2=2 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walk.py \
  tests/test_gpu_multi.py tests/test_gpu_chunked.py -x -q --timeout 240 --timeout-method thread > "$OUT/tests.log" 2>&1 \
  || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for rep in 1 2 3; do
  for e in 2 1 0; do
    CVD_JIT_DEFINES=-DCVD_BS_ETAB2=$e timeout -k 10 300 python3 bench.py --cpu-baseline 0 --early-decision 0 --steps 6 --warmup 1 \
      > "$OUT/sweep_etab${e}_$rep.json" 2> "$OUT/sweep_etab${e}_$rep.err" || { tail -5 "$OUT/sweep_etab${e}_$rep.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/sweep_etab${e}_$rep.json').read().strip().splitlines()[-1]);print('etab=$e rep=$rep',round(d['value']),[round(x['ms']) for x in d['diagnostic']['detector_ms_by_launch']])"
  done
done
