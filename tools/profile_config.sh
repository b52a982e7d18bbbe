#!/bin/bash
# Kernel stats + HBM traffic + VALU/LDS counts of one bench configuration (run on the GPU box):
#   bash tools/profile_config.sh <tag> <config> [steps]      e.g. r02_c5_v1 c5 2
# -> gpurun_out/<tag>/{stats,pmc_fetch,pmc_write,valu}/ ; summarise on the CPU side with
#    python tools/traffic_summary.py gpurun_out/<tag> <tag>  and  python tools/pmc_table.py
set -e
TAG=$1
CFG=${2:-c4}
STEPS=${3:-5}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --config $CFG --no-cpu --no-e2e --no-pmc"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
  python $B --steps $STEPS --warmup 1 > $OUT/stats.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
  python $B --steps 1 --warmup 1 > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
  python $B --steps 1 --warmup 1 > $OUT/pmc_write.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  --output-format csv -d $OUT/valu -o run -- python $B --steps 1 --warmup 1 > $OUT/valu.log 2>&1
echo done
