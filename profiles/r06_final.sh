#!/bin/bash
# Round 6 evidence of record: the GPU suite + smoke(), the driver's exact command, the same
# command under rocprofv3 --kernel-trace --stats, and the per-p PMC passes (one counter group
# per pass, never with a trace domain) that profiles/summarize.py turns into
# profiles/pmc_markov_m6.json.
#   bash profiles/r06_final.sh gpurun_out/r06m
set -uo pipefail
OUT=${1:?out dir}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
bash profiles/run_gpu_tests.sh "$OUT" || exit 1
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver_cmd.json" 2> "$OUT/bench_driver_cmd.err" \
  || { tail "$OUT/bench_driver_cmd.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench_driver_cmd.json').read().strip().splitlines()[-1]);print('driver cmd',round(d['value']),round(d['roofline']['avg_launch_ms'],2),d['cpu_baseline']['value'],d['reference_call']['second_call_s'])"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$ROOT/$OUT/trace" -o run \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err" || { tail "$OUT/bench_trace.err"; exit 1; }
echo "trace done"
ARGS="--config m6 --cpu-baseline 0 --early-decision 0 --steps 6 --warmup 0"
i=0
for grp in "FETCH_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 600 rocprofv3 --pmc $grp -T --output-format csv -d "$ROOT/$OUT/pmc$i" -o run \
    -- python3 bench.py $ARGS > "$OUT/bench_pmc$i.json" 2>/dev/null || exit 1
  echo "pass $i done"
done
