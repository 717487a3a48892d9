#!/bin/bash
# rehearse the driver's 8-rank run on the one card before it happens.
# 8 ranks (gloo, CVD_BENCH_ONE_DEVICE=1: all on device 0; RCCL needs one GPU per rank)
# with an EMPTY JIT cache and no model cache: 8 concurrent clang compiles and 8 x 6 GPU
# model builds.  Then one rank over the same global trial ids (8 x the batch): the
# per-p counts must be equal.
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
export CVD_JIT_CACHE=$(mktemp -d /tmp/cvd_jit_empty.XXXXXX)
unset CVD_MODEL_CACHE
B=4096
common="--config m6 --steps 2 --warmup 1 --cpu-baseline 0"
CVD_BENCH_ONE_DEVICE=1 timeout -k 10 600 python bench.py --gpus 8 --dist-backend gloo --batch $B $common > $OUT/r8.json 2> $OUT/r8.err || { echo "8-rank run failed"; tail -20 $OUT/r8.err; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --batch $((8 * B)) $common > $OUT/r1.json 2> $OUT/r1.err || { tail -20 $OUT/r1.err; exit 1; }
python - $OUT <<'PY'
import json, sys
o = sys.argv[1]
j8 = json.loads(open(o + "/r8.json").read().strip().splitlines()[-1])
j1 = json.loads(open(o + "/r1.json").read().strip().splitlines()[-1])
eq = j8["diagnostic"]["per_p"] == j1["diagnostic"]["per_p"]
res = {"n_gpus_8": j8["n_gpus"], "n_gpus_1": j1["n_gpus"], "per_p_equal": eq,
       "setup_by_rank": j8["diagnostic"]["setup_by_rank"],
       "early_counts_equal": j8.get("early_decision", {}).get("counts_equal_full_run"),
       "value_8_ranks_one_card": j8["value"], "value_1": j1["value"]}
print(json.dumps(res, indent=1))
json.dump(res, open(o + "/rehearse8_summary.json", "w"), indent=1)
sys.exit(0 if eq and j8["n_gpus"] == 8 else 1)
PY
