#!/bin/bash
# Round-3 GPU call (rewritten per call; git history keeps each version).  Usage: bash tools/gpu_r03.sh <tag>
# v14: each buffer set's analysis on its own high-priority stream (FRA_DUAL_ANA) -- parity (pipeline tests
# incl. set_raster), A/B dual vs single on C4 x3, C3 x3, C5, and the SGPR-capped build (co-resident
# background k_minmax_vec) with dual streams.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|error" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
D=$GRAFT_REPO_ROOT/flac-raster_amd/flac_raster/_lib/diag
run() {  # lib dual cfg
  FRA_LIB_PATH=$1 FRA_DUAL_ANA=$2 timeout -k 10 300 python -u bench.py --config $3 --no-cpu --no-e2e --no-pmc --no-trace > $OUT/b.json 2> $OUT/b.err || { echo BENCH_FAILED $1 $2 $3; tail -20 $OUT/b.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-4s %-6s dual=%s %10.1f MPix/s %8.4f ms/step' % ('$3', '$(basename "$1" .so | sed s/libflac_raster_amd_exp_//)', '$2', d['value'], d['ms_per_step']), r['kernel_ms_per_launch'])" | tee -a $OUT/ab.txt
}
for rep in 1 2 3; do
  for cfg in c4 c3; do
    run "" 1 $cfg; run "" 0 $cfg; run $D/libflac_raster_amd_exp_cap94.so 1 $cfg
  done
done
run "" 1 c5; run "" 0 c5
echo ALLOK
