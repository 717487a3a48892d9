set -uo pipefail
mkdir -p gpurun_out/r06ah
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_walk.py tests/test_gpu_multi.py tests/test_gpu_chunked.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r06ah/tests.log 2>&1 || { tail -30 gpurun_out/r06ah/tests.log; exit 1; }
tail -1 gpurun_out/r06ah/tests.log
bash profiles/r06_walk01.sh gpurun_out/r06ag && bash profiles/r04_rehearse8.sh gpurun_out/r06af
