#!/bin/bash
# Round-5 HEAD lines: GPU suite + smoke, the driver's default bench command (C4 with CPU, e2e and PMC legs),
# C3 and C5 lines (C5 with the bounded-memory ring e2e leg), then the frame-split shard projections:
# bash tools/gpu_r05_final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r05_final}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --prof-dir $OUT/prof_c4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo BENCH_FAILED c4; tail -20 $OUT/bench_c4.err; exit 1; }
tail -c 400 $OUT/bench_c4.json
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --config c3 --no-cpu --prof-dir $OUT/prof_c3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo BENCH_FAILED c3; tail -20 $OUT/bench_c3.err; exit 1; }
tail -c 300 $OUT/bench_c3.json
timeout -k 10 900 python3 bench.py --gpus 1 --steps 10 --warmup 3 --config c5 --no-cpu --prof-dir $OUT/prof_c5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo BENCH_FAILED c5; tail -20 $OUT/bench_c5.err; exit 1; }
tail -c 300 $OUT/bench_c5.json
for S in ${SHARDS:-0/2 1/2 0/4 3/4 0/8 7/8}; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 30 --warmup 5 --config c4 --shard $S --no-cpu --no-e2e --no-pmc >> $OUT/shard.jsonl 2>> $OUT/shard.err || { echo SHARD_FAILED c4 $S; tail -20 $OUT/shard.err; exit 1; }
  tail -1 $OUT/shard.jsonl
done
for S in ${SHARDS5:-0/8 7/8}; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 10 --warmup 3 --config c5 --shard $S --no-cpu --no-e2e --no-pmc >> $OUT/shard.jsonl 2>> $OUT/shard.err || { echo SHARD_FAILED c5 $S; tail -20 $OUT/shard.err; exit 1; }
  tail -1 $OUT/shard.jsonl
done
echo ALLOK
