#!/bin/bash
# VALU instruction mix + LDS detail of k_analyze on the C4 workload (one rocprofv3 PMC pass per group)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
i=0
for CTRS in "SQ_WAVES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64" \
            "SQ_WAVES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VALU" \
            "SQ_WAVES SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/p$i -o run -- \
    python $GRAFT_REPO_ROOT/tools/diag_phases.py ${LIB:--} > $OUT/p$i.log 2>&1 || echo "pass $i failed" >> $OUT/fail.log
done
echo done
