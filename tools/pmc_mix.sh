#!/bin/bash
# VALU instruction mix, LDS detail, issue / I-cache counters of the analysis on the C4 workload (one rocprofv3
# PMC pass per group).  usage: LIB=<lib.so> bash tools/pmc_mix.sh <out> ; then tools/pmc_table.py <out> <kernel>
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
i=0
for CTRS in "SQ_WAVES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64" \
            "SQ_WAVES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VALU" \
            "SQ_WAVES SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES" \
            "SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU" \
            "SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/p$i -o run -- \
    python $GRAFT_REPO_ROOT/tools/diag_phases.py ${LIB:--} ${CFG:-c4} > $OUT/p$i.log 2>&1 || echo "pass $i failed" >> $OUT/fail.log
done
echo done
