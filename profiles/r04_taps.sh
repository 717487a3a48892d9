#!/bin/bash
# Round 4: unrolled encoder tap lists (ChunkEncoder kT > 0) -- stream parity, then
# generator-alone A/B (tap lists / CVD_GEN_TAP_LOOP=1 / the per-phase rate-2/3 build
# lib/libcvd_old23.so), the C3 and C1 lines both ways, and C4
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
L=detecting-convolutional-codes-via-markovian-statistics_amd/lib
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_gen_taps.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_grid.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  for c in r23_m4 m6; do
    timeout -k 10 120 python profiles/gen_only.py $c 5 > $OUT/gen_${c}_lists_$i.txt 2>&1 || exit 1
    CVD_GEN_TAP_LOOP=1 timeout -k 10 120 python profiles/gen_only.py $c 5 > $OUT/gen_${c}_loop_$i.txt 2>&1 || exit 1
  done
  GEN_ONLY_LIB=$PWD/$L/libcvd_old23.so timeout -k 10 120 python profiles/gen_only.py r23_m4 5 > $OUT/gen_r23_m4_old23_$i.txt 2>&1 || exit 1
done
tail -n 4 $OUT/gen_*.txt
summ() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],round(d['value']),'ms/step',round(d['ms_per_step'],2),'gen',round(d['diagnostic'].get('generator_ms_per_step',0),2),'det',round(d['diagnostic'].get('detector_ms_per_step',0),2))" $1; }
for v in lists loop; do
  E=""; [ $v = loop ] && E="CVD_GEN_TAP_LOOP=1"
  env $E timeout -k 10 300 python bench.py --config r23_m4 --cpu-baseline 0 --early-decision 0 > $OUT/bench_r23_$v.json 2> $OUT/bench_r23_$v.err || { tail -5 $OUT/bench_r23_$v.err; exit 1; }
  summ $OUT/bench_r23_$v.json
  env $E timeout -k 10 300 python bench.py --config m2 --cpu-baseline 0 --early-decision 0 > $OUT/bench_m2_$v.json 2> $OUT/bench_m2_$v.err || { tail -5 $OUT/bench_m2_$v.err; exit 1; }
  summ $OUT/bench_m2_$v.json
done
timeout -k 10 900 python -u bench.py --config c4 --cpu-baseline 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -5 $OUT/bench_c4.err; exit 1; }
tail -c 600 $OUT/bench_c4.json
