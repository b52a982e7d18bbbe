#!/bin/bash
# Round-4 HEAD lines: the driver's default bench command (C4 with CPU, e2e and PMC legs), then C3 and C5
# lines with counters, then the shard projections: bash tools/gpu_r04_final2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04_final2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo BENCH_FAILED c4; tail -20 $OUT/bench_c4.err; exit 1; }
tail -c 400 $OUT/bench_c4.json
for CFG in c3 c5; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --config $CFG --no-cpu --no-e2e > $OUT/bench_$CFG.json 2> $OUT/bench_$CFG.err || { echo BENCH_FAILED $CFG; tail -20 $OUT/bench_$CFG.err; exit 1; }
  tail -c 300 $OUT/bench_$CFG.json
done
bash tools/gpu_r04_shard.sh ${1:-r04_final2}_shard c4 c3 c5
