#!/bin/bash
# round 3, GPU call 3: device rows numbered by learning-chain visits (hot rows together)
# -- parity tests, interleaved A/B against first-visit order over the sweep's p
set -uo pipefail
mkdir -p gpurun_out/r03c
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_bfs.py \
  tests/test_gpu_learn.py tests/test_gpu_early.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03c/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/r03c/tests.log; exit 1; }
tail -2 gpurun_out/r03c/tests.log
timeout -k 10 400 python -u profiles/ab_k1b.py --variant= "--variant=;CVD_ROW_ORDER=first" --p 0.01 0.02 0.05 0.1 0.2 \
  --rounds 3 --out gpurun_out/r03c/ab_roworder.jsonl > gpurun_out/r03c/ab.log 2>&1 || { echo "AB FAILED"; tail -20 gpurun_out/r03c/ab.log; exit 1; }
grep median gpurun_out/r03c/ab.log | python3 -c "import sys,json; [print(json.loads(l)['p'], json.loads(l)['median']) for l in sys.stdin]"
echo ALL DONE
