#!/bin/bash
# r02 v26: 16-bit lag-12 k_analyze (levels 7-8) at 5 waves/SIMD (95 VGPRs, no scratch) -- parity at level 8 + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02_v26}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_direct_write.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
L=flac-raster_amd/flac_raster/_lib/ab
for i in 1 2 3; do
  for lib in libA libB; do
    timeout -k 10 200 python -u tools/diag_phases.py $L/$lib.so c4 8 >> $OUT/ab.txt 2>&1 || { echo AB_FAILED; tail -20 $OUT/ab.txt; exit 1; }
  done
done
for lib in libA libB; do
  timeout -k 10 200 python -u tools/diag_phases.py $L/$lib.so c3 7 >> $OUT/ab.txt 2>&1 || { echo AB_FAILED; tail -20 $OUT/ab.txt; exit 1; }
done
grep -v Warning $OUT/ab.txt | grep lib
echo ALLOK
