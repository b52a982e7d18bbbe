#!/bin/bash
# background-grid experiment: bench step time by FRA_BG_BLOCKS (0 = full grid)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-bgexp}
mkdir -p $OUT
for nb in 256 64 128 512 0 256; do
  FRA_BG_BLOCKS=$nb timeout -k 10 200 python -u bench.py --no-cpu --no-e2e --no-pmc > $OUT/bench_$nb.json 2> $OUT/bench_$nb.err || { echo BENCH_FAILED; tail -30 $OUT/bench_$nb.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_$nb.json').read().strip().splitlines()[-1]); print('bg', $nb, d['value'], d['ms_per_step'])"
done
FRA_PIPE=0 timeout -k 10 200 python -u bench.py --no-cpu --no-e2e --no-pmc > $OUT/bench_nopipe.json 2> $OUT/bench_nopipe.err || { echo BENCH_FAILED; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_nopipe.json').read().strip().splitlines()[-1]); print('nopipe', d['value'], d['ms_per_step'])"
echo ALLOK
