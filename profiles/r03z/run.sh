#!/bin/bash
# round 3: filter pattern table of 1,024 entries (8 KiB) against 4,096 (32 KiB), global filter,
# the lockstep p of the sweep (the host build and the JIT kernel use the same table size; run
# on the tree before commit bfbbee3, where CVD_FILTER_PAT_BITS was a host env knob and a JIT define)
set -uo pipefail
O=gpurun_out/r03z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u profiles/ab_k1b.py --variant= --variant="-DCVD_FILTER_PAT_BITS=12;CVD_FILTER_PAT_BITS=12" \
  --p 0.05 0.1 0.2 --rounds 3 --out $O/ab_pat.jsonl > $O/ab_pat.log 2>&1 || { echo "AB FAILED"; tail -20 $O/ab_pat.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r03z/ab_pat.jsonl"):
    d = json.loads(l); print(d["p"], {k: round(v, 1) for k, v in d["median"].items()})
PY
