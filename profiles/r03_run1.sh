#!/bin/bash
# round 3, GPU call 1: the GPU test suite + smoke on the round's first tree, then the
# sweep-wide rocprofv3 evidence (trace + per-p PMC) for m6, m2 and r23_m4
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03a_gputests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -30 gpurun_out/r03a_gputests.log; exit 1; }
tail -3 gpurun_out/r03a_gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03a_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/r03a_smoke.log; exit 1; }
tail -1 gpurun_out/r03a_smoke.log
for cfg in ${CFGS:-m6 m2 r23_m4}; do
  bash profiles/collect_sweep.sh gpurun_out/r03a_$cfg $cfg || { echo "COLLECT $cfg FAILED"; exit 1; }
done
echo ALL DONE
