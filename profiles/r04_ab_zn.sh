#!/bin/bash
# A/B of the zero-test toggle (CVD_K1B_ZN_CHAIN) in one process, identical sums required
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python profiles/ab_k1b.py --variant= --variant=-DCVD_K1B_ZN_CHAIN=1 --p 0.01 0.05 0.1 0.2 --rounds 3 --out $OUT/ab_zn.jsonl > $OUT/ab_zn.log 2>&1 || { tail -20 $OUT/ab_zn.log; exit 1; }
cat $OUT/ab_zn.jsonl
