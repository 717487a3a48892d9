#!/bin/bash
# round 3 evidence, part 3 (walk mode in the tree): the driver's headline command, the
# C1 / C3 lines, smoke, and C4 on one GPU
set -uo pipefail
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err \
  || { echo "BENCH FAILED"; tail -20 $O/bench_default.err; exit 1; }
echo "default done" >&2
timeout -k 10 300 python -u bench.py --config m2 > $O/bench_m2.json 2> $O/bench_m2.err || { echo "M2 FAILED"; exit 1; }
timeout -k 10 300 python -u bench.py --config r23_m4 > $O/bench_r23_m4.json 2> $O/bench_r23_m4.err || { echo "R23 FAILED"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; exit 1; }
timeout -k 10 900 python -u bench.py --config c4 > $O/bench_c4.json 2> $O/bench_c4.err || { echo "C4 FAILED"; exit 1; }
echo ALL DONE
