#!/bin/bash
# Round-4 GPU check: GPU suite, smoke(), then a bench line (C4 by default, no CPU/e2e legs unless FULL=1).
# usage: bash tools/gpu_r04.sh <tag> [config]
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04}
CFG=${2:-c4}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
EXTRA="--no-cpu --no-e2e"
[ "$FULL" = 1 ] && EXTRA=""
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --config $CFG $EXTRA > $OUT/bench_$CFG.json 2> $OUT/bench_$CFG.err || { echo BENCH_FAILED; tail -20 $OUT/bench_$CFG.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_$CFG.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('kernel_ms_per_launch'))"
echo ALLOK
