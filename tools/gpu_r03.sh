#!/bin/bash
# Round-3 GPU call (rewritten per call; git history keeps each version).  Usage: bash tools/gpu_r03.sh <tag>
# v15: k_analyze phase stamps at HEAD (coarse and fine: the load phase split into metadata / raw loads / LUT
# gathers / LDS + reductions / barrier), C4 and C3.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for cfg in c4 c3; do
  timeout -k 10 200 python -u tools/stamp_phases.py $cfg > $OUT/stamps_$cfg.txt 2>&1 || { echo STAMPS_FAILED $cfg; tail $OUT/stamps_$cfg.txt; exit 1; }
  timeout -k 10 200 python -u tools/stamp_phases.py $cfg --fine > $OUT/stamps_fine_$cfg.txt 2>&1 || { echo FINE_FAILED $cfg; tail $OUT/stamps_fine_$cfg.txt; exit 1; }
done
cat $OUT/stamps_c4.txt $OUT/stamps_fine_c4.txt $OUT/stamps_fine_c3.txt
echo ALLOK
