#!/bin/bash
# A/B of the rate-2/3 generator: stride-3 encoder (lib/libcvd.so) against the per-phase
# windows (lib/libcvd_old23.so, built with -DCVD_GEN_K2_STRIDE3=0), generator alone
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
L=detecting-convolutional-codes-via-markovian-statistics_amd/lib
for i in 1 2; do
  timeout -k 10 120 python profiles/gen_only.py r23_m4 5 > $OUT/new_$i.txt 2>&1 || exit 1
  GEN_ONLY_LIB=$PWD/$L/libcvd_old23.so timeout -k 10 120 python profiles/gen_only.py r23_m4 5 > $OUT/old_$i.txt 2>&1 || exit 1
done
timeout -k 10 120 python profiles/gen_only.py m6 5 > $OUT/m6_new.txt 2>&1 || exit 1
tail -n 4 $OUT/*.txt
# C4 with the workspace allocated before the timed region
timeout -k 10 900 python -u bench.py --config c4 --cpu-baseline 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -5 $OUT/bench_c4.err; exit 1; }
tail -c 600 $OUT/bench_c4.json
