#!/bin/bash
# shard projection (bench.py --shard R/N: one GPU runs the heaviest LPT rank's share) + the 1-GPU lines of
# the same configs, same box: bash tools/gpu_r04_shard.sh <tag> [configs...]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for CFG in ${@:-c4 c3}; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --config $CFG --no-cpu --no-e2e --no-pmc > $OUT/n1_$CFG.json 2> $OUT/n1_$CFG.err || { echo BENCH_FAILED $CFG; tail -20 $OUT/n1_$CFG.err; exit 1; }
  tail -1 $OUT/n1_$CFG.json
  SH="0/2 0/4 4/8"
  [ $CFG != c4 ] && SH="0/8"
  for S in $SH; do
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 30 --warmup 5 --config $CFG --shard $S --no-cpu --no-e2e --no-pmc >> $OUT/shard.jsonl 2>> $OUT/shard.err || { echo SHARD_FAILED $CFG $S; tail -20 $OUT/shard.err; exit 1; }
    tail -1 $OUT/shard.jsonl
  done
done
echo ALLOK
