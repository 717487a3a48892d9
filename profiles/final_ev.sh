#!/bin/bash
# Round-end evidence: every GPU test, smoke(), the three bench configs, the default
# bench line (CPU baseline, Pd match, early decision), then the rocprofv3 trace + PMC.
set -uo pipefail
OUT=$1; export TMPDIR=/tmp
bash profiles/quick_gpu.sh $OUT || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
python -c "import json;d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]);print('default',d['value'],d['cpu_baseline']['value'],d['pd_match_vs_cpu']['match'])"
bash profiles/collect.sh ${OUT}_prof
