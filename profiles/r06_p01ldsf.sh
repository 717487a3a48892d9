#!/bin/bash
# Round 6: p = 0.01 -- walk + LDS filter (default before), lockstep + pre-filter (CVD_WALK=0),
# lockstep + LDS filter (CVD_WALK=0 CVD_LDSF_LOCKSTEP=1): sums, then two alternating rounds.
#   bash profiles/r06_p01ldsf.sh gpurun_out/r06ai
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 profiles/r06_p01modes.py > "$OUT/modes.txt" 2>&1 || { tail -20 "$OUT/modes.txt"; exit 1; }
cat "$OUT/modes.txt"
for rep in 1 2; do
  for m in walk lockpf lockldsf; do
    case $m in walk) E="X=1";; lockpf) E="CVD_WALK=0";; lockldsf) E="CVD_WALK=0 CVD_LDSF_LOCKSTEP=1";; esac
    env $E timeout -k 10 180 python3 bench.py --cpu-baseline 0 --early-decision 0 --p 0.01 --steps 3 --warmup 1 \
      > "$OUT/p01_${m}_$rep.json" 2> "$OUT/p01_${m}_$rep.err" || { tail -5 "$OUT/p01_${m}_$rep.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/p01_${m}_$rep.json').read().strip().splitlines()[-1]);print('p=0.01 $m',round(d['roofline']['avg_launch_ms'],1))"
  done
done
for m in lockpf lockldsf; do
  case $m in lockpf) E="CVD_WALK=0";; lockldsf) E="CVD_WALK=0 CVD_LDSF_LOCKSTEP=1";; esac
  env $E timeout -k 10 180 python3 bench.py --cpu-baseline 0 --early-decision 0 --p 0.02 --steps 3 --warmup 1 \
    > "$OUT/p02_${m}.json" 2> "$OUT/p02_${m}.err" || { tail -5 "$OUT/p02_${m}.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/p02_${m}.json').read().strip().splitlines()[-1]);print('p=0.02 $m',round(d['roofline']['avg_launch_ms'],1))"
done
