#!/bin/bash
# r02 v29: one cross-queue wait per pipelined execute on the plan's stream (A/B: FRA_PACK_WAIT=1 = old)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02_v29}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for cfg in c4 c3; do
  for w in 1 0 1 0; do
    FRA_PACK_WAIT=$w timeout -k 10 300 python -u bench.py --config $cfg --no-cpu --no-e2e --no-pmc > $OUT/${cfg}_$w.json 2> $OUT/${cfg}_$w.err || { echo BENCH_FAILED; tail -20 $OUT/${cfg}_$w.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/${cfg}_$w.json').read().strip().splitlines()[-1]); print('$cfg packwait=$w', d['value'], d['ms_per_step'])" | tee -a $OUT/summary.txt
  done
done
echo ALLOK
