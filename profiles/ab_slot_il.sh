set -uo pipefail
OUT=gpurun_out/r02z5_il; mkdir -p $OUT; export TMPDIR=/tmp
CVD_SLOT_IL=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/tests_il.log 2>&1 || { tail -20 $OUT/tests_il.log; exit 1; }
tail -1 $OUT/tests_il.log
for v in 0 1 1 0; do
  CVD_SLOT_IL=$v timeout -k 10 300 python bench.py --cpu-baseline 0 --early-decision 0 > $OUT/m6_il$v.$RANDOM.json 2>/dev/null || exit 1
done
python - <<'P'
import json,glob
for f in sorted(glob.glob('gpurun_out/r02z5_il/m6_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, round(d['value']), {k:round(v) for k,v in d['diagnostic']['detector_ms_by_p'].items()})
P
