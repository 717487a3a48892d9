#!/bin/bash
# round 3 final tree: evidence pass, the driver's bench command, and the m6 sweep PMC
set -uo pipefail
bash profiles/run_evidence.sh gpurun_out/r03fin || exit 1
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r03fin/bench_driver_cmd.json 2> gpurun_out/r03fin/bench_driver_cmd.err || exit 1
bash profiles/collect_sweep.sh gpurun_out/r03fin_m6 m6 || exit 1
