set -uo pipefail
mkdir -p gpurun_out/r04z
timeout -k 10 300 python profiles/bitslice_acs_run.py 16667 262144 > gpurun_out/r04z/bitslice.txt 2>&1; rc=$?
cat gpurun_out/r04z/bitslice.txt | tail -5
exit $rc
