#!/bin/bash
# Detector PMC at single grid points (bench.py --p): how the per-wave-step VALU
# and the wait fractions move with p.   bash profiles/pmc_by_p.sh gpurun_out/pmcp "0.01 0.1"
set -uo pipefail
export TMPDIR=/tmp
O=$PWD/$1; PS=${2:-"0.01 0.1"}
mkdir -p $O
for p in $PS; do
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "FETCH_SIZE"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp -T --output-format csv -d $O/p${p}_g$i -o run \
      -- python3 bench.py --p $p --steps 1 --warmup 0 --cpu-baseline 0 --early-decision 0 > $O/p${p}_g$i.json 2>$O/p${p}_g$i.err || exit 1
  done
  echo "p=$p done"
done
