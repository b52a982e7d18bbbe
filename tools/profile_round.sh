#!/bin/bash
# One round's measurement set (run on the GPU box from the repo root):
#   bash tools/profile_round.sh <tag>        e.g. r01_c4_n1_v8
# 1. python bench.py (default C4 line, CPU baseline + e2e)              -> gpurun_out/<tag>/bench.json
# 2. rocprofv3 --kernel-trace --stats on bench.py (kernels only)          -> gpurun_out/<tag>/stats/
# 3. rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE (separate passes) -> gpurun_out/<tag>/pmc_{fetch,write}/
# Then on the CPU side: python tools/traffic_summary.py gpurun_out/<tag> <tag>
set -e
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python $GRAFT_REPO_ROOT/bench.py > $OUT/bench.json 2> $OUT/bench.err
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --no-cpu --no-e2e --steps 20 --warmup 3 > $OUT/stats.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --no-cpu --no-e2e --steps 3 --warmup 1 > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --no-cpu --no-e2e --steps 3 --warmup 1 > $OUT/pmc_write.log 2>&1
echo done
