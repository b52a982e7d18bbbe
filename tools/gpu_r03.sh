#!/bin/bash
# Round-3 GPU call (rewritten per call; git history keeps each version).  Usage: bash tools/gpu_r03.sh <tag>
# v12: L2 prefetch extended to the 32-bit path (FRA_PREFETCH32 = 1024) -- parity, A/B against a build
# without any prefetch on C5 (x2) and C4.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|error" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
D=flac-raster_amd/flac_raster/_lib/diag
run() {  # lib-or-empty tag cfg
  FRA_LIB_PATH=$1 timeout -k 10 300 python -u bench.py --config $3 --no-cpu --no-e2e --no-pmc --no-trace > $OUT/b.json 2> $OUT/b.err || { echo BENCH_FAILED $2 $3; tail -20 $OUT/b.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-4s %-7s %10.1f MPix/s %8.4f ms/step' % ('$3', '$2', d['value'], d['ms_per_step']), r['kernel_ms_per_launch'])" | tee -a $OUT/ab.txt
}
for rep in 1 2; do
  run "" pf c5; run $GRAFT_REPO_ROOT/$D/libflac_raster_amd_exp_pf0.so pf0 c5
done
run "" pf c4; run $GRAFT_REPO_ROOT/$D/libflac_raster_amd_exp_pf0.so pf0 c4
echo ALLOK
