#!/bin/bash
# round 3: key compare with one subtraction per word and bitop3 pairs (CVD_K1B_CMPX) A/B;
# walk schedule thresholds at p = 0.01 / 0.02 with two-step records
set -uo pipefail
O=gpurun_out/r03o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u profiles/ab_k1b.py --variant= --variant=-DCVD_K1B_CMPX=1 --p 0.01 0.05 0.1 0.2 \
  --rounds 3 --out $O/ab_cmpx.jsonl > $O/ab_cmpx.log 2>&1 || { echo "AB CMPX FAILED"; tail -20 $O/ab_cmpx.log; exit 1; }
tail -4 $O/ab_cmpx.log
timeout -k 10 400 python -u profiles/ab_k1b.py --variant= --variant=";CVD_WALK_WMIN=40" --variant=";CVD_WALK_WMIN=56" \
  --variant=";CVD_WALK_AMIN=4" --variant=";CVD_WALK_AMIN=16" --p 0.01 0.02 \
  --rounds 3 --out $O/ab_sched.jsonl > $O/ab_sched.log 2>&1 || { echo "AB SCHED FAILED"; tail -20 $O/ab_sched.log; exit 1; }
tail -2 $O/ab_sched.log
echo ALL DONE
