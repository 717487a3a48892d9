#!/bin/bash
# GPU-box pass: the -m gpu suite (one process, per-test timeout) and smoke().
#   bash profiles/run_gpu_tests.sh gpurun_out/t [extra pytest args]
set -uo pipefail
OUT=${1:-gpurun_out/t}
shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "$@" \
  > "$OUT/gpu_tests.log" 2>&1
rc=$?
tail -5 "$OUT/gpu_tests.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
tail -2 "$OUT/smoke.log"
