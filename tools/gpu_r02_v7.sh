#!/bin/bash
# r02 v7: the default bench line (C4: CPU baselines, e2e, in-run PMC) + rocprofv3 kernel stats of C4 and C5
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02_v7
mkdir -p $OUT
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/stats_c4 -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --config c4 --no-cpu --no-e2e --no-pmc --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/$OUT/stats_c4.log 2>&1 || { echo STATS_C4_FAILED; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/stats_c5 -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --config c5 --no-cpu --no-e2e --no-pmc --steps 5 --warmup 1 > $GRAFT_REPO_ROOT/$OUT/stats_c5.log 2>&1 || { echo STATS_C5_FAILED; exit 1; }
tail -1 $GRAFT_REPO_ROOT/$OUT/stats_c4.log
tail -1 $GRAFT_REPO_ROOT/$OUT/stats_c5.log
echo ALLOK
