#!/bin/bash
# A/B of k1s variants on the headline sweep (run on the GPU box from the repo root):
#   bash profiles/r05_ab.sh OUTDIR "NAME1:ENV1" "NAME2:ENV2" ...
# each variant: one bench.py run (--steps 6: one launch per p), env as given
# (e.g. "pat11w5:CVD_BS_PAT_BITS=11 CVD_JIT_DEFINES=-DCVD_K1B_WAVES=5"); BENCH_ARGS adds bench
# options (e.g. BENCH_ARGS="--p 0.01" STEPS=3: one p)
set -uo pipefail
OUT=${1:?out dir}; shift
mkdir -p "$OUT"
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  echo "variant $name: $envs" >&2
  env $envs timeout -k 10 400 python -u bench.py --steps ${STEPS:-6} --warmup 1 --cpu-baseline 0 --early-decision 0 ${BENCH_ARGS:-} \
    > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" || { echo "variant $name failed" >&2; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$OUT/bench_$name.json').read().strip().split('\n')[-1])
print('$name', round(d['value']), [(x['p'][0], round(x['ms'])) for x in d['diagnostic']['detector_ms_by_launch']])
" | tee -a "$OUT/summary.txt"
done
