#!/bin/bash
# Round 4: generator slot lanes compute the sequence ids (2 KB of LDS per block) against
# the LDS copy (CVD_GEN_SEQ_LDS=1 build, lib/libcvd_seqlds.so): stream parity, generator
# alone, the C3 line (overlapped with the detector, where LDS decides co-residency)
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/detecting-convolutional-codes-via-markovian-statistics_amd/lib
PT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_gen_taps.py tests/test_gpu_parity.py -k "generator or tap" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -n 1 $OUT/tests.log
summ() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],round(d['value']),'ms/step',round(d['ms_per_step'],2),'gen',round(d['diagnostic'].get('generator_ms_per_step',0),2),'det',round(d['diagnostic'].get('detector_ms_per_step',0),2))" $1; }
B="python bench.py --cpu-baseline 0 --early-decision 0"
for i in 1 2; do
  for v in default seqlds; do
    E="CVD_NOP=1"; [ $v = seqlds ] && E="CVD_LIB_PATH=$L/libcvd_seqlds.so"
    env $E timeout -k 10 120 python profiles/gen_only.py r23_m4 5 > $OUT/gen_r23_$v.$i.txt 2>&1 || exit 1
    env $E timeout -k 10 300 $B --config r23_m4 > $OUT/bench_r23_$v.$i.json 2> $OUT/bench_r23_$v.$i.err || { tail -5 $OUT/bench_r23_$v.$i.err; exit 1; }
    summ $OUT/bench_r23_$v.$i.json
  done
done
tail -n 2 $OUT/gen_*.txt
