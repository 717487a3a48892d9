#!/bin/bash
# Round 4: generator encoder tap lists (ChunkEncoder kT > 0) and the split noise exchange
# (CVD_GEN_XCHG_SPLIT) -- stream parity, then generator-alone A/B (default / tap loop
# CVD_GEN_TAP_LOOP=1 / unsplit exchange lib/libcvd_xold.so / per-phase rate-2/3
# lib/libcvd_old23.so), the C3 and C1 lines (C1 also with the split exchange in the fused
# kernel, lib/libcvd_fsplit.so), and C4
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/detecting-convolutional-codes-via-markovian-statistics_amd/lib
PT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_gen_taps.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_grid.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
CVD_LIB_PATH=$L/libcvd_fsplit.so timeout -k 10 300 $PT tests/test_gpu_fused.py > $OUT/tests_fsplit.log 2>&1 || { tail -30 $OUT/tests_fsplit.log; exit 1; }
tail -1 $OUT/tests_fsplit.log
for i in 1 2; do
  for c in r23_m4 m6; do
    timeout -k 10 120 python profiles/gen_only.py $c 5 > $OUT/gen_${c}_default_$i.txt 2>&1 || exit 1
    CVD_GEN_TAP_LOOP=1 timeout -k 10 120 python profiles/gen_only.py $c 5 > $OUT/gen_${c}_taploop_$i.txt 2>&1 || exit 1
    CVD_LIB_PATH=$L/libcvd_xold.so timeout -k 10 120 python profiles/gen_only.py $c 5 > $OUT/gen_${c}_xold_$i.txt 2>&1 || exit 1
  done
  CVD_LIB_PATH=$L/libcvd_old23.so timeout -k 10 120 python profiles/gen_only.py r23_m4 5 > $OUT/gen_r23_m4_old23_$i.txt 2>&1 || exit 1
done
tail -n 4 $OUT/gen_*.txt
summ() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],round(d['value']),'ms/step',round(d['ms_per_step'],2),'gen',round(d['diagnostic'].get('generator_ms_per_step',0),2),'det',round(d['diagnostic'].get('detector_ms_per_step',0),2))" $1; }
B="python bench.py --cpu-baseline 0 --early-decision 0"
for v in default taploop xold; do
  case $v in default) E="CVD_NOP=1";; taploop) E="CVD_GEN_TAP_LOOP=1";; xold) E="CVD_LIB_PATH=$L/libcvd_xold.so";; esac
  env $E timeout -k 10 300 $B --config r23_m4 > $OUT/bench_r23_$v.json 2> $OUT/bench_r23_$v.err || { tail -5 $OUT/bench_r23_$v.err; exit 1; }
  summ $OUT/bench_r23_$v.json
done
for v in default taploop fsplit; do
  case $v in default) E="CVD_NOP=1";; taploop) E="CVD_GEN_TAP_LOOP=1";; fsplit) E="CVD_LIB_PATH=$L/libcvd_fsplit.so";; esac
  env $E timeout -k 10 300 $B --config m2 > $OUT/bench_m2_$v.json 2> $OUT/bench_m2_$v.err || { tail -5 $OUT/bench_m2_$v.err; exit 1; }
  summ $OUT/bench_m2_$v.json
done
timeout -k 10 300 $B --config r23_m4 --fused 1 > $OUT/bench_r23_fused.json 2> $OUT/bench_r23_fused.err || { tail -5 $OUT/bench_r23_fused.err; exit 1; }
summ $OUT/bench_r23_fused.json
timeout -k 10 900 python -u bench.py --config c4 --cpu-baseline 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -5 $OUT/bench_c4.err; exit 1; }
tail -c 600 $OUT/bench_c4.json
