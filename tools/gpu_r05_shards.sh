#!/bin/bash
# every rank's share of an N-way split, one GPU, one bench line each (bench.py --shard r/N --split S):
# CFG=c4 N=8 SPLITS="frames strided" bash tools/gpu_r05_shards.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r05_shards}
mkdir -p $OUT
export TMPDIR=/tmp
N=${N:-8}
for S in ${SPLITS:-frames strided}; do
  for R in $(seq 0 $((N - 1))); do
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 30 --warmup 5 --config ${CFG:-c4} --shard $R/$N --split $S \
      --no-cpu --no-e2e --no-pmc >> $OUT/shard.jsonl 2>> $OUT/shard.err || { echo SHARD_FAILED $S $R; tail -20 $OUT/shard.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['split'], d['shard'], d['tiles'], d['frames'], d['ms_per_step'], d['kernel_ms_per_launch']['analyze'])" $OUT/shard.jsonl
  done
done
echo ALLOK
