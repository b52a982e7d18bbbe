#!/bin/bash
# r02 v15 (re-entry check): GPU test suite, default bench line, rocprofv3 kernel stats of the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r02_v15
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --no-cpu --no-e2e --no-pmc --steps 20 --warmup 3 > $OUT/stats.log 2>&1 || { echo STATS_FAILED; tail -20 $OUT/stats.log; exit 1; }
echo ALLOK
