#!/bin/bash
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -5 $OUT/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1; rc=$?
tail -2 $OUT/smoke.log
exit $rc
