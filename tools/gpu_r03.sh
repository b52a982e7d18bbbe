#!/bin/bash
# Round-3 GPU call (rewritten per call; git history keeps each version).  Usage: bash tools/gpu_r03.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 120 python -u tools/stamp_phases.py c4 --fine > $OUT/stamps_c4_fine.txt 2>&1 || { echo STAMP_FAILED; tail -20 $OUT/stamps_c4_fine.txt; exit 1; }
cat $OUT/stamps_c4_fine.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 600 python -u bench.py --config c4 --no-cpu --no-e2e --prof-dir $OUT/prof > $OUT/c4.json 2> $OUT/c4.err || { echo C4_FAILED; tail -20 $OUT/c4.err; exit 1; }
echo ALLOK
