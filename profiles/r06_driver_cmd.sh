#!/bin/bash
# Round 6: the driver's exact bench command at the tree's HEAD (plus the GPU suite when asked).
#   bash profiles/r06_driver_cmd.sh gpurun_out/r06a [tests]
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${2:-}" = "tests" ]; then
  bash profiles/run_gpu_tests.sh "$OUT" || exit 1
fi
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver_cmd.json" 2> "$OUT/bench_driver_cmd.err" \
  || { tail "$OUT/bench_driver_cmd.err"; exit 1; }
python3 - "$OUT/bench_driver_cmd.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"], "launch ms", d["roofline"]["avg_launch_ms"],
      "cpu", d.get("cpu_baseline", {}).get("value"), "ref_call", d.get("reference_call", {}).get("second_call_s"))
print("box", json.dumps(d.get("box"))[:600])
PY
