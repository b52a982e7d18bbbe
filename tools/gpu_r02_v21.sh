#!/bin/bash
# r02 v21 (HEAD c55bf38+): full default bench line (PMC roofline, CPU baselines, e2e), rocprofv3 kernel
# stats of the same workload, all five configurations
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02_v21}
mkdir -p $OUT
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-600
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --no-cpu --no-e2e --no-pmc --steps 20 --warmup 3 > $OUT/stats.log 2>&1 || { echo STATS_FAILED; tail -20 $OUT/stats.log; exit 1; }
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u tools/bench_configs.py --out $OUT/configs.json > $OUT/configs.log 2>&1 || { echo CONFIGS_FAILED; tail -20 $OUT/configs.log; exit 1; }
grep -v Warning $OUT/configs.log | cut -c1-300 | tail -8
echo ALLOK
