#!/bin/bash
# round 3: walk mode with block jobs (one H1 block per CU, k1b_body): parity tests, then A/B
# against the static H1/H2 wave interleave and lockstep
set -uo pipefail
O=gpurun_out/r03r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_walk.py -x -v --timeout 240 --timeout-method thread > $O/walk_tests.log 2>&1 \
  || { echo "WALK TESTS FAILED"; tail -30 $O/walk_tests.log; exit 1; }
tail -1 $O/walk_tests.log
timeout -k 10 500 python -u profiles/ab_k1b.py --variant= --variant=";CVD_WALK_H1_PER_CU=0" --variant=";CVD_WALK_H1_PER_CU=2" \
  --variant=";CVD_WALK=0" --p 0.01 0.02 --rounds 2 --out $O/ab_jobs.jsonl > $O/ab_jobs.log 2>&1 \
  || { echo "AB FAILED"; tail -20 $O/ab_jobs.log; exit 1; }
timeout -k 10 500 python -u profiles/ab_k1b.py --variant=";CVD_WALK=1" --variant=";CVD_WALK=0" --p 0.05 0.1 \
  --rounds 2 --out $O/ab_jobs_hi.jsonl > $O/ab_jobs_hi.log 2>&1 || { echo "AB HI FAILED"; tail -20 $O/ab_jobs_hi.log; exit 1; }
python3 - <<'PY'
import json
for f in ["gpurun_out/r03r/ab_jobs.jsonl", "gpurun_out/r03r/ab_jobs_hi.jsonl"]:
    for l in open(f):
        d = json.loads(l); print(d["p"], {k: round(v, 1) for k, v in d["median"].items()})
PY
