#!/bin/bash
# Round 6: prebuilt JIT test, the 8-rank rehearsal (empty user JIT cache), C4 in full.
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit_variants.py -x -v --timeout 300 --timeout-method thread \
  > "$OUT/tests_jit.log" 2>&1 || { tail -20 "$OUT/tests_jit.log"; exit 1; }
tail -3 "$OUT/tests_jit.log"
bash profiles/r04_rehearse8.sh "$OUT/rehearse8" > "$OUT/rehearse8.log" 2>&1 || { tail -20 "$OUT/rehearse8.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/rehearse8/rehearse8_summary.json'));print('setup',[round(x['setup_s'],1) for x in d['setup_by_rank']],d['per_p_equal'])"
timeout -k 10 900 python3 bench.py --config c4 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" || { tail -5 "$OUT/bench_c4.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench_c4.json').read().strip().splitlines()[-1]);print('c4',round(d['value']),{k:round(v['trials_per_s']) for k,v in d['per_N'].items()}, {k:round(v['seconds'],1) for k,v in d['per_N'].items()})"
