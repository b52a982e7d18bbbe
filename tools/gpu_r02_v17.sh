#!/bin/bash
# r02 v17 (re-entry baseline at HEAD): full GPU suite, default bench line, rocprofv3 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02_v17}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --no-cpu --no-e2e --no-pmc --steps 20 --warmup 3 > $OUT/stats.log 2>&1 || { echo STATS_FAILED; tail -20 $OUT/stats.log; exit 1; }
echo ALLOK
