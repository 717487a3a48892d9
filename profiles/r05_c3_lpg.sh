#!/bin/bash
# C3's table detector with only the 16-bit records and log T_ref in LDS
# and log P̂1 gathered from global memory (cvd_kernels.hip LdsModel kLpG, CVD_T16_LPG=1;
# 256-thread blocks, 29 KB of LDS instead of 145 KB) against the default LDS image: bench
# lines and one rocprofv3 kernel trace each (GPU box, repo root):
#   bash profiles/r05_c3_lpg.sh OUTDIR
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in 0 1; do
  CVD_T16_LPG=$v timeout -k 10 300 python -u bench.py --config r23_m4 --steps 20 --warmup 3 --cpu-baseline 0 \
    --early-decision 0 > "$OUT/bench_lpg$v.json" 2> "$OUT/bench_lpg$v.err" || { echo "bench lpg=$v failed" >&2; exit 1; }
  CVD_T16_LPG=$v timeout -s KILL 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace_lpg$v" -o run \
    -- python3 bench.py --config r23_m4 --steps 4 --warmup 1 --cpu-baseline 0 --early-decision 0 \
    > "$OUT/trace_lpg$v.json" 2> "$OUT/trace_lpg$v.err" || { echo "trace lpg=$v failed" >&2; exit 1; }
  python3 - "$OUT" "$v" <<'EOF' | tee -a "$OUT/summary.txt"
import csv, glob, json, sys
out, v = sys.argv[1], sys.argv[2]
d = json.loads(open(f"{out}/bench_lpg{v}.json").read().strip().split("\n")[-1])
st = {}
for f in glob.glob(f"{out}/trace_lpg{v}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        st[r["Name"][:60]] = round(float(r["AverageNs"]) / 1e6, 3)
print(json.dumps({"lpg": int(v), "trials_per_s": d["value"], "ms_per_step": d["ms_per_step"], "kernel_avg_ms": st}))
EOF
done
