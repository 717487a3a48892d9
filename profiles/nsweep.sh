#!/bin/bash
# Single-GPU leg of BASELINE config C4: the m = 6 pair over N = 1e3 .. 1e6 (bench.py --N).
#   bash profiles/nsweep.sh gpurun_out/nsweep
set -uo pipefail
OUT=${1:-gpurun_out/nsweep}
mkdir -p "$OUT"
for N in 1000 10000 1000000; do
  if [ $N -eq 1000000 ]; then ARGS="--batch 262144 --steps 2 --warmup 1"; else ARGS="--steps 6"; fi
  timeout -k 10 600 python bench.py --N $N $ARGS --cpu-baseline 0 --early-decision 0 > "$OUT/bench_N$N.json" || exit 1
  python -c "import json;d=json.loads(open('$OUT/bench_N$N.json').read().strip().splitlines()[-1]);print($N, d['value'], d['diagnostic']['detector_ms_per_step'], d['diagnostic']['generator_ms_per_step'])"
done
