#!/bin/bash
# r02 v23: nontemporal slot stores (k_analyze) + slot loads / frame stores (k_assemble), same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02_v23}
mkdir -p $OUT
L=flac-raster_amd/flac_raster/_lib/ab
timeout -k 10 600 bash tools/gpu_ab.sh $L/libA.so $L/libB.so c4 3 > $OUT/ab_c4.txt 2>&1 || { echo AB_FAILED; tail -20 $OUT/ab_c4.txt; exit 1; }
grep -v Warning $OUT/ab_c4.txt | grep "lib"
timeout -k 10 600 bash tools/gpu_ab.sh $L/libA.so $L/libB.so c3 2 > $OUT/ab_c3.txt 2>&1 || { echo AB_FAILED; tail -20 $OUT/ab_c3.txt; exit 1; }
grep -v Warning $OUT/ab_c3.txt | grep "lib"
echo ALLOK
