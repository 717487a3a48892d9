#!/bin/bash
# C1's fused kernel with kCp interleaved copies of its LDS image
# (cvd_kernels.hip LdsModel, CVD_C1_COPIES) against the single image: the bench line of each
# and one rocprofv3 --pmc pass of the LDS counters per variant (GPU box, repo root):
#   bash profiles/r05_c1_copies.sh OUTDIR [COPIES...]
set -uo pipefail
OUT=${1:?out dir}; shift
CPS=${@:-1 4 8 16}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cp in $CPS; do
  CVD_C1_COPIES=$cp timeout -k 10 300 python -u bench.py --config m2 --steps 10 --warmup 2 --cpu-baseline 0 \
    --early-decision 0 > "$OUT/bench_cp$cp.json" 2> "$OUT/bench_cp$cp.err" || { echo "bench cp=$cp failed" >&2; exit 1; }
  CVD_C1_COPIES=$cp timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
    -T --output-format csv -d "$OUT/pmc_cp$cp" -o run -- python3 bench.py --config m2 --steps 1 --warmup 0 \
    --cpu-baseline 0 --early-decision 0 > "$OUT/pmc_cp$cp.json" 2> "$OUT/pmc_cp$cp.err" || { echo "pmc cp=$cp failed" >&2; exit 1; }
  python3 - "$OUT" "$cp" <<'EOF' | tee -a "$OUT/summary.txt"
import csv, glob, json, sys
out, cp = sys.argv[1], sys.argv[2]
d = json.loads(open(f"{out}/bench_cp{cp}.json").read().strip().split("\n")[-1])
tot = {}
for f in glob.glob(f"{out}/pmc_cp{cp}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mc_table16" in r.get("Kernel_Name", ""):
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
c = tot.get("SQ_LDS_BANK_CONFLICT", 0.0); a = tot.get("SQ_LDS_IDX_ACTIVE", 0.0)
print(json.dumps({"copies": int(cp), "trials_per_s": d["value"], "ms_per_step": d["ms_per_step"],
                  "lds_bank_conflict_frac_of_active": c / a if a else None, "counters": tot}))
EOF
done
