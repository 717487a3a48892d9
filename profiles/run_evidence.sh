#!/bin/bash
# One GPU-box pass of the round's evidence (run from the repo root via gpurun):
# GPU parity tests, smoke(), the bench line for every BASELINE config that fits one
# GPU, and a rocprofv3 kernel-trace/stats pass of the headline bench.
#   bash profiles/run_evidence.sh gpurun_out/ev
set -uo pipefail
OUT=${1:-gpurun_out/ev}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > "$OUT/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -3 "$OUT/gpu_tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
timeout -k 10 600 python bench.py > "$OUT/bench_m6.json" 2> "$OUT/bench_m6.err" || exit 1
timeout -k 10 600 python bench.py --config m2 > "$OUT/bench_m2.json" 2> "$OUT/bench_m2.err" || exit 1
timeout -k 10 600 python bench.py --config r23_m4 > "$OUT/bench_r23_m4.json" 2> "$OUT/bench_r23_m4.err" || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$ROOT/$OUT/trace" -o run \
  -- python3 bench.py --cpu-baseline 0 --early-decision 0 > "$OUT/bench_under_rocprof.json" || exit 1
echo "evidence collected in $OUT"
