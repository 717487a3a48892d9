#!/bin/bash
# Round 6: which pipe the lockstep m = 6 launch (p = 0.05) keeps busy -- texture address / data
# (TA / TD), the vector L1 (TCP), LDS and VALU -- one --pmc pass per run, each under its own limit.
#   bash profiles/r06_pmc_pipe.sh gpurun_out/r06v
set -uo pipefail
OUT=${1:?out dir}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || echo "counter list failed"
ARGS="--cpu-baseline 0 --early-decision 0 --p ${P:-0.05} --steps 1 --warmup 0"
i=0
for grp in "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD" \
           "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "MemUnitBusy" "VALUBusy"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp -T --output-format csv -d "$ROOT/$OUT/pmc$i" -o run \
    -- python3 bench.py $ARGS > "$OUT/pmc$i.json" 2> "$OUT/pmc$i.err"
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pass $i ($grp) failed rc=$rc"; tail -3 "$OUT/pmc$i.err"
    case $rc in 124|134|137|139) exit $rc;; esac   # (a kill, abort or fault ends the call)
    continue
  fi
  echo "pass $i ($grp) done"
done
