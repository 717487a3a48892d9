#!/bin/bash
# Round 6: the walk's compact 8-B two-step records (value table in LDS) against the 32-B records
# (CVD_WALK_T2C=0 at model build): the walk suite, then p = 0.01 launches and the headline.
#   bash profiles/r06_t2c.sh gpurun_out/r06p
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py -x -q --timeout 240 --timeout-method thread \
  > "$OUT/tests_walk.log" 2>&1 || { tail -20 "$OUT/tests_walk.log"; exit 1; }
tail -1 "$OUT/tests_walk.log"
for rep in 1 2; do for t in 0 1; do
  CVD_WALK_T2C=$t timeout -k 10 150 python3 bench.py --cpu-baseline 0 --early-decision 0 --p 0.01 --steps 3 --warmup 1 \
    > "$OUT/p01_t2c${t}_$rep.json" 2> "$OUT/p01_t2c${t}_$rep.err" || { tail -5 "$OUT/p01_t2c${t}_$rep.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/p01_t2c${t}_$rep.json').read().strip().splitlines()[-1]);print('p=0.01 t2c=$t',round(d['roofline']['avg_launch_ms'],1))"
done; done
for t in 0 1; do
  CVD_WALK_T2C=$t timeout -k 10 150 python3 bench.py --cpu-baseline 0 --early-decision 0 --steps 6 --warmup 1 \
    > "$OUT/hl_t2c$t.json" 2> "$OUT/hl_t2c$t.err" || { tail -5 "$OUT/hl_t2c$t.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/hl_t2c$t.json').read().strip().splitlines()[-1]);print('headline t2c=$t',round(d['value']),[round(x['ms'],1) for x in d['diagnostic']['detector_ms_by_launch']])"
done
