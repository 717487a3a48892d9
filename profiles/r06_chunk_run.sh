#!/bin/bash
# Round 6: the chunked detector's GPU tests and the reference-call timing.
#   bash profiles/r06_chunk_run.sh gpurun_out/r06b
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_chunked.py -x -v --timeout 240 --timeout-method thread \
  > "$OUT/tests_chunked.log" 2>&1
rc=$?
tail -15 "$OUT/tests_chunked.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 profiles/r06_refcall.py > "$OUT/refcall.json" 2> "$OUT/refcall.err" || { tail "$OUT/refcall.err"; exit 1; }
cat "$OUT/refcall.err"
python3 -c "import json;d=json.load(open('$OUT/refcall.json'));print(d['dataframes_equal'])"
