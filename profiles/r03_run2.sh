#!/bin/bash
# round 3, GPU call 2: the 64-bit lazy key compare (CVD_K1B_CMP64) -- parity tests, an
# interleaved A/B against the word-by-word compare over the sweep's p, and the GPU BFS
# of the m = 6 decoder (state count or certified lower bound, 300 s budget)
set -uo pipefail
mkdir -p gpurun_out/r03b
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_jit_variants.py \
  -x -v --timeout 300 --timeout-method thread > gpurun_out/r03b/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/r03b/tests.log; exit 1; }
tail -2 gpurun_out/r03b/tests.log
timeout -k 10 300 python -u profiles/ab_k1b.py --variant= --variant=-DCVD_K1B_CMP64=0 --p 0.01 0.05 0.1 0.2 \
  --out gpurun_out/r03b/ab_cmp64.jsonl > gpurun_out/r03b/ab.log 2>&1 || { echo "AB FAILED"; tail -20 gpurun_out/r03b/ab.log; exit 1; }
cat gpurun_out/r03b/ab.log | grep median | python3 -c "import sys,json; [print(json.loads(l)['p'], json.loads(l)['median']) for l in sys.stdin]"
CVD_BFS_VERBOSE=1 CVD_BFS_SECONDS=300 timeout -k 10 420 python -u profiles/bfs_m6.py gpurun_out/r03b/bfs_m6.json \
  > gpurun_out/r03b/bfs.log 2>&1 || { echo "BFS FAILED"; tail -20 gpurun_out/r03b/bfs.log; exit 1; }
tail -5 gpurun_out/r03b/bfs.log
echo ALL DONE
