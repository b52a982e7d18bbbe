#!/bin/bash
# r02 v20: wave index in SGPRs (no scratch in the 7-wave 16-bit k_analyze) -- parity + same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02_v20}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_direct_write.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
L=flac-raster_amd/flac_raster/_lib/ab
timeout -k 10 600 bash tools/gpu_ab.sh $L/libA.so $L/libB.so c4 3 > $OUT/ab_c4.txt 2>&1 || { echo AB_FAILED; tail -20 $OUT/ab_c4.txt; exit 1; }
grep -v Warning $OUT/ab_c4.txt | grep "lib"
timeout -k 10 600 bash tools/gpu_ab.sh $L/libA.so $L/libB.so c5 1 > $OUT/ab_c5.txt 2>&1 || { echo AB_FAILED; tail -20 $OUT/ab_c5.txt; exit 1; }
grep -v Warning $OUT/ab_c5.txt | grep "lib"
echo ALLOK
