#!/bin/bash
# round 3: LDS filter (512 threads, 64 KiB, walking models <= 32,768 rows) against the global
# filter at full launch size, then the evidence pass
set -uo pipefail
O=gpurun_out/r03x3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u profiles/ab_k1b.py --trials 2621440 --variant= --variant=";CVD_NO_LDSF=1" --p 0.01 0.02 \
  --rounds 2 --out $O/ab_ldsf_full.jsonl > $O/ab_ldsf_full.log 2>&1 || { echo "AB FAILED"; tail -20 $O/ab_ldsf_full.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r03x3/ab_ldsf_full.jsonl"):
    d = json.loads(l); print(d["p"], {k: round(v, 1) for k, v in d["median"].items()})
PY
bash profiles/run_evidence.sh gpurun_out/r03y
