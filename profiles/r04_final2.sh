#!/bin/bash
# Round 4 final evidence at HEAD, part 1: the whole GPU suite and smoke(), then the
# driver's bench command (CPU baseline, Pd match, C0) and the m2 / r23 lines.
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -n 2 $OUT/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver_cmd.json 2> $OUT/bench_driver_cmd.err || { tail -20 $OUT/bench_driver_cmd.err; exit 1; }
timeout -k 10 300 python bench.py --config m2 > $OUT/bench_m2.json 2> $OUT/bench_m2.err || { tail -20 $OUT/bench_m2.err; exit 1; }
timeout -k 10 300 python bench.py --config r23_m4 > $OUT/bench_r23_m4.json 2> $OUT/bench_r23_m4.err || { tail -20 $OUT/bench_r23_m4.err; exit 1; }
python -c "
import json
for f in ['bench_driver_cmd','bench_m2','bench_r23_m4']:
    d=json.loads(open('$OUT/'+f+'.json').read().strip().splitlines()[-1])
    print(f, round(d['value']), d.get('value_wall'), d['roofline'].get('frac'), (d.get('cpu_baseline') or {}).get('value'), (d.get('pd_match_vs_cpu') or {}).get('match'), (d.get('c0_demo') or {}).get('match'), d['diagnostic'].get('generator_ms_per_step'), d['diagnostic'].get('detector_ms_per_step'))
"
