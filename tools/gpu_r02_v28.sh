#!/bin/bash
# r02 v28: background norm-stage grid size (FRA_BG_BLOCKS) on C5 and C4
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02_v28}
mkdir -p $OUT
for cfg in c5 c4; do
  for bg in 256 128 512 1024 256; do
    FRA_BG_BLOCKS=$bg timeout -k 10 300 python -u bench.py --config $cfg --no-cpu --no-e2e --no-pmc > $OUT/${cfg}_$bg.json 2> $OUT/${cfg}_$bg.err || { echo BENCH_FAILED; tail -20 $OUT/${cfg}_$bg.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/${cfg}_$bg.json').read().strip().splitlines()[-1]); print('$cfg bg=$bg', d['value'], d['ms_per_step'])" | tee -a $OUT/summary.txt
  done
done
echo ALLOK
