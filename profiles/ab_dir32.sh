#!/bin/bash
# Directory load 1/32 vs the default 1/16 (one bench.py --p launch per point).
set -uo pipefail
OUT=${1:-gpurun_out/r02z19_dir32}; mkdir -p $OUT; export TMPDIR=/tmp
for p in 0.1 0.05 0.2; do
  for v in 4 5 4; do
    CVD_DIR_LOAD_LOG2=$v timeout -k 10 300 python bench.py --cpu-baseline 0 --early-decision 0 --p $p --steps 3 --warmup 1 > $OUT/l$v.p$p.$RANDOM.json 2>/dev/null || exit 1
  done
done
python - <<'P'
import json,glob
for f in sorted(glob.glob('gpurun_out/r02z19_dir32/*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f.split('/')[-1], round(d['diagnostic']['detector_ms_per_step'],1), round(d['diagnostic']['model_setup_s'],2))
P
