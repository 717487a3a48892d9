#!/bin/bash
# what bounds the dense-table kernels (C1: the fused mc_table16_kernel;
# C3: detect_table16_kernel) -- LDS instruction, bank-conflict and LDS-wait counters beside
# VALU, one rocprofv3 --pmc pass per group (<= 8 SQ + 1 GRBM counters each).
set -uo pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -o "SQ_[A-Z_]*LDS[A-Z_]*\|SQ_INST_CYCLES_[A-Z_]*\|SQ_ACTIVE_INST_[A-Z_]*\|SQ_INSTS_[A-Z_]*" $OUT/avail.txt | sort -u > $OUT/sq_lds_counters.txt || true
cat $OUT/sq_lds_counters.txt | tr '\n' ' '; echo
for cfg in m2 r23_m4; do
  i=0
  for grp in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $grp -T --output-format csv -d "$OUT/${cfg}_pmc$i" -o run \
      -- python3 bench.py --config $cfg --steps 1 --warmup 0 --cpu-baseline 0 --early-decision 0 --multi 0 > "$OUT/${cfg}_pmc$i.json" 2> "$OUT/${cfg}_pmc$i.err" || { echo "pass $cfg $i failed"; tail -5 "$OUT/${cfg}_pmc$i.err"; exit 1; }
    echo "pass $cfg $i done"
  done
done
