#!/bin/bash
# pipelined min/max grid A/B on C5 (alternating) and on the C4 8-way / 4-way shares: bash tools/gpu_r04_mmgrid.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for V in 1 0; do
    for S in 4/8 0/4; do
      FRA_MM_PER_CU=$V timeout -k 10 300 python3 bench.py --gpus 1 --steps 30 --warmup 5 --config c4 --shard $S --no-cpu --no-e2e --no-pmc > $OUT/s.json 2>> $OUT/shard.err || { echo SHARD_FAILED; tail -20 $OUT/shard.err; exit 1; }
      echo "per_cu=$V $(tail -1 $OUT/s.json)" >> $OUT/shard.txt
    done
  done
done
bash tools/gpu_r04_abs.sh $TAG c5 "- FRA_MM_PER_CU=1" "- FRA_MM_PER_CU=0" > /dev/null
echo ALLOK
