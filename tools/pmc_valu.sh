#!/bin/bash
# VALU issue accounting of k_analyze on the C4 workload (one rocprofv3 PMC pass):
#   bash tools/pmc_valu.sh <tag>   -> gpurun_out/<tag>/valu/   (summarise: python tools/pmc_table.py)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
  --output-format csv -d $OUT/valu -o run -- python $GRAFT_REPO_ROOT/tools/diag_phases.py > $OUT/valu.log 2>&1
echo done
