#!/bin/bash
# round 3: directory load factor at the walking p (smaller directory: fewer Infinity-Cache
# misses on the H2 waves' row hits, longer probes)
set -uo pipefail
O=gpurun_out/r03ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u profiles/ab_k1b.py --trials 2621440 --variant= --variant=";CVD_DIR_LOAD_LOG2=3" \
  --variant=";CVD_DIR_LOAD_LOG2=2" --variant=";CVD_DIR_LOAD_LOG2=5" --p 0.01 0.02 \
  --rounds 1 --out $O/ab_dirload.jsonl > $O/ab_dirload.log 2>&1 || { echo "AB FAILED"; tail -20 $O/ab_dirload.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/r03ab/ab_dirload.jsonl"):
    d = json.loads(l); print(d["p"], {k: round(v, 1) for k, v in d["median"].items()})
PY
