#!/bin/bash
# Filter sizing: words >= rows (default) vs words >= rows / 2 (CVD_FILTER_SCALE=-1), cap 2 MiB.
set -uo pipefail
OUT=${1:-gpurun_out/r02z11_filt}; mkdir -p $OUT; export TMPDIR=/tmp
for p in 0.01 0.02 0.05 0.15; do
  for v in 0 -1; do
    CVD_FILTER_SCALE=$v timeout -k 10 300 python bench.py --cpu-baseline 0 --early-decision 0 --p $p --steps 3 --warmup 1 > $OUT/s$v.p$p.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads(open('$OUT/s$v.p$p.json').read().strip().splitlines()[-1]);print('scale $v','p=$p',round(d['diagnostic']['detector_ms_per_step'],1), d['config']['model_rows_p0'])"
  done
done
