#!/bin/bash
# Stall / issue breakdown of k_analyze (full build) on the C4 workload: one rocprofv3 PMC pass per
# counter group (no trace domains combined with --pmc).  Usage (GPU box, repo root):
#   bash tools/pmc_stalls.sh <out-subdir>
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY" \
            "SQ_WAVES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_WAIT_INST_LDS" \
            "SQ_WAVES SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/p$i -o run -- \
    python $GRAFT_REPO_ROOT/tools/diag_phases.py ${LIB:--} > $OUT/p$i.log 2>&1 || echo "pass $i failed" >> $OUT/fail.log
done
echo done
