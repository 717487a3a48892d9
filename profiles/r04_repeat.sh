#!/bin/bash
# Round 4: a second HEAD sample of the driver's bench command and the C3 line (run-to-run spread)
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver_cmd.err || { tail -20 $OUT/bench_driver_cmd.err; exit 1; }
timeout -k 10 300 python bench.py --config r23_m4 > $OUT/bench_r23_m4.json 2> $OUT/bench_r23_m4.err || { tail -20 $OUT/bench_r23_m4.err; exit 1; }
timeout -k 10 300 python bench.py --config m2 > $OUT/bench_m2.json 2> $OUT/bench_m2.err || { tail -20 $OUT/bench_m2.err; exit 1; }
python -c "
import json
for f in ['bench_driver_cmd','bench_r23_m4','bench_m2']:
    d=json.loads(open('$OUT/'+f+'.json').read().strip().splitlines()[-1])
    print(f, round(d['value']), d.get('value_wall'), (d.get('pd_match_vs_cpu') or {}).get('match'), (d.get('c0_demo') or {}).get('match'))
"
