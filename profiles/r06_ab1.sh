#!/bin/bash
# Round 6 A/Bs: (1) the headline with the chunked instantiation compiled out vs in (same
# sums; the unchunked loop's code must not lose), (2) C4's N = 1e6 launches chunked vs not,
# (3) --sweep all chunked vs not.
#   bash profiles/r06_ab1.sh gpurun_out/r06d
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="--cpu-baseline 0 --early-decision 0"
run() { # name, env..., -- args
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py $B ${ARGS} > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -5 "$OUT/$name.err"; exit 1; }
  python3 - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pn = d.get("per_N")
extra = {k: round(v["trials_per_s"]) for k, v in pn.items()} if pn else [round(x["ms"], 1) for x in d["diagnostic"]["detector_ms_by_launch"]]
print(sys.argv[2], round(d["value"]), extra, flush=True)
PY
}
ARGS="--steps 6 --warmup 1"
run hl_ck_out CVD_JIT_DEFINES=-DCVD_K1S_CK=0 CVD_CHUNK=0
run hl_default CVD_CHUNK=-1
run hl_ck_out2 CVD_JIT_DEFINES=-DCVD_K1S_CK=0 CVD_CHUNK=0
run hl_default2 CVD_CHUNK=-1
ARGS="--config c4 --c4-N 1000000 --c4-trials 786432 --p 0.05"
run c4_n1e6_p05_unchunked CVD_CHUNK=0
run c4_n1e6_p05_chunked CVD_CHUNK=-1
ARGS="--config c4 --c4-N 1000000 --c4-trials 786432 --p 0.2"
run c4_n1e6_p20_unchunked CVD_CHUNK=0
run c4_n1e6_p20_chunked CVD_CHUNK=-1
ARGS="--sweep all --steps 2 --warmup 1"
run sweepall_unchunked CVD_CHUNK=0
run sweepall_chunked CVD_CHUNK=-1
