#!/bin/bash
# Round 6: directory slots of three 128-B lines, each {two phase images,
# the record} (CVD_BS_SLOT3=1), against the 256-B slots: sums (GPU suites under the variant),
# the headline A/B on one box, and FETCH_SIZE per launch at p = 0.05 / 0.1.
#   bash profiles/r06_slot3.sh gpurun_out/r06j
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
CVD_BS_SLOT3=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walk.py tests/test_gpu_multi.py \
  tests/test_gpu_chunked.py -x -q --timeout 240 --timeout-method thread > "$OUT/tests_slot3.log" 2>&1 \
  || { tail -20 "$OUT/tests_slot3.log"; exit 1; }
tail -1 "$OUT/tests_slot3.log"
B="--cpu-baseline 0 --early-decision 0 --steps 6 --warmup 1"
for rep in 1 2; do for s3 in 0 1; do
  CVD_BS_SLOT3=$s3 timeout -k 10 300 python3 bench.py $B > "$OUT/hl_s${s3}_$rep.json" 2> "$OUT/hl_s${s3}_$rep.err" || { tail -5 "$OUT/hl_s${s3}_$rep.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/hl_s${s3}_$rep.json').read().strip().splitlines()[-1]);print('slot3=$s3',round(d['value']),[round(x['ms'],1) for x in d['diagnostic']['detector_ms_by_launch']])"
done; done
for p in 0.05 0.1; do for s3 in 0 1; do
  CVD_BS_SLOT3=$s3 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$ROOT/$OUT/pmc_p${p}_s$s3" -o run \
    -- python3 bench.py --p $p --steps 1 --warmup 0 --cpu-baseline 0 --early-decision 0 > "$OUT/pmc_p${p}_s$s3.json" 2>/dev/null || exit 1
  python3 - "$OUT/pmc_p${p}_s$s3" "$p" "$s3" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "k1b" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
v = sum(float(r["Counter_Value"]) for r in rows) * 1024
alg = 2_621_440 * 2 * 25_000
print(f"p={sys.argv[2]} slot3={sys.argv[3]} FETCH raw {v/1e12:.3f} TB per launch, x alg (raw + stream half) {(v + alg/2)/alg:.1f}")
PY
done; done
