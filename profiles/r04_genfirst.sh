#!/bin/bash
# (Round 4 A/B; the CVD_BENCH_GEN_FIRST knob was removed from bench.py after it measured neutral)
set -uo pipefail
OUT=$1; mkdir -p $OUT; export TMPDIR=/tmp
summ() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],round(d['value']),'ms/step',round(d['ms_per_step'],2),'gen',round(d['diagnostic'].get('generator_ms_per_step',0),2),'det',round(d['diagnostic'].get('detector_ms_per_step',0),2))" $1; }
B="python bench.py --cpu-baseline 0 --early-decision 0 --config r23_m4"
for i in 1 2; do for g in 0 1; do
  CVD_BENCH_GEN_FIRST=$g timeout -k 10 300 $B > $OUT/bench_r23_gf$g.$i.json 2> $OUT/bench_r23_gf$g.$i.err || { tail -5 $OUT/bench_r23_gf$g.$i.err; exit 1; }
  summ $OUT/bench_r23_gf$g.$i.json
done; done
