#!/bin/bash
# Round-3 GPU call (rewritten per call; git history keeps each version).  Usage: bash tools/gpu_r03.sh <tag>
# v24: the HEAD measurement set (product build after the v22/v23 A/Bs were dropped): full GPU suite,
# the default C4 bench line (all legs), C3 and C5 with counters + timed kernel stats, the shard projections.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
export FRA_PROF_DIR=$OUT/prof
timeout -k 10 420 python -u bench.py > $OUT/c4.json 2> $OUT/c4.err || { echo BENCH_C4_FAILED; tail -20 $OUT/c4.err; exit 1; }
for cfg in c3 c5; do
timeout -k 10 420 python -u bench.py --config $cfg --no-cpu --no-e2e > $OUT/$cfg.json 2> $OUT/$cfg.err || { echo BENCH_FAILED $cfg; tail -20 $OUT/$cfg.err; exit 1; }
done
unset FRA_PROF_DIR
for cfg in c4 c3 c5; do
python -c "import json; d=json.loads(open('$OUT/$cfg.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg', d['value'], d['ms_per_step'], r['kernel_ms_per_launch'], r['frac'], r['valu_issue_frac'], (r['counters'] or {}).get('stalls'))"
done
for sh in c4:0/2 c4:0/4 c4:4/8 c3:0/8 c5:0/8; do
  cfg=${sh%%:*}; r=${sh#*:}
  timeout -k 10 300 python -u bench.py --config $cfg --shard $r --no-cpu --no-e2e --no-pmc --no-trace > $OUT/shard.json 2> $OUT/shard.err || { echo SHARD_FAILED $sh; tail -20 $OUT/shard.err; exit 1; }
  tail -1 $OUT/shard.json >> $OUT/shard.txt
done
echo ALLOK
