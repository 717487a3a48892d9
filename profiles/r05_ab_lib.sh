#!/bin/bash
# A/B of library builds (ahead-of-time kernels, e.g. the generator) on the headline bench, run
# alternately on one GPU box from the repo root:
#   bash profiles/r05_ab_lib.sh OUTDIR ROUNDS "NAME1:LIBPATH1" "NAME2:LIBPATH2" ...
# (CVD_LIB_PATH selects the library; BENCH_ARGS adds bench options)
set -uo pipefail
OUT=${1:?out dir}; ROUNDS=${2:-2}; shift 2
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    name=${v%%:*}; lib=${v#*:}
    CVD_LIB_PATH="$lib" timeout -k 10 400 python -u bench.py --steps ${STEPS:-6} --warmup 1 --cpu-baseline 0 --early-decision 0 ${BENCH_ARGS:-} \
      > "$OUT/bench_${name}_$r.json" 2> "$OUT/bench_${name}_$r.err" || { echo "variant $name failed" >&2; exit 1; }
    python3 -c "
import json
d=json.loads(open('$OUT/bench_${name}_$r.json').read().strip().split('\n')[-1])
dg=d['diagnostic']
print('$name', $r, round(d['value']), 'gen', round(dg.get('generator_ms_per_step') or 0, 1), [(x['p'][0], round(x['ms'])) for x in dg.get('detector_ms_by_launch', [])])
" | tee -a "$OUT/summary.txt"
  done
done
