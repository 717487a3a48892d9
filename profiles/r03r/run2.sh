#!/bin/bash
# round 3: block jobs at full launch size (2,621,440 trials), and per-wave job traces
set -uo pipefail
O=gpurun_out/r03r2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u profiles/ab_k1b.py --trials 2621440 --variant= --variant=";CVD_WALK_H1_PER_CU=0" \
  --variant=";CVD_WALK_H1_PER_CU=2" --variant=";CVD_WALK_H1_PER_CU=3" --p 0.01 0.02 --rounds 1 \
  --out $O/ab_jobs_full.jsonl > $O/ab_jobs_full.log 2>&1 || { echo "AB FAILED"; tail -20 $O/ab_jobs_full.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r03r2/ab_jobs_full.jsonl"):
    d = json.loads(l); print(d["p"], {k: round(v, 1) for k, v in d["median"].items()})
PY
timeout -k 10 400 python -u profiles/ab_k1b.py --trials 2621440 \
  --variant="-DCVD_JOB_TRACE=1;CVD_WALK_H1_PER_CU=1;CVD_JOB_TRACE_FILE=$O/trace1.bin" \
  --variant="-DCVD_JOB_TRACE=1;CVD_WALK_H1_PER_CU=2;CVD_JOB_TRACE_FILE=$O/trace2.bin" \
  --p 0.01 --rounds 1 > $O/trace.log 2>&1 || { echo "TRACE FAILED"; tail -20 $O/trace.log; exit 1; }
ls -la $O
