#!/bin/bash
# Round-3 GPU call (rewritten per call; git history keeps each version).  Usage: bash tools/gpu_r03.sh <tag>
# v18: fine k_analyze stamps with per-role finish times (Levinson-Durbin wave vs the two FIXED-search
# waves inside the LD phase; the LPC partition-search wave), C4 and C3.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for cfg in c4 c3; do
  timeout -k 10 200 python -u tools/stamp_phases.py $cfg --fine > $OUT/stamps_fine_$cfg.txt 2>&1 || { echo FINE_FAILED $cfg; tail $OUT/stamps_fine_$cfg.txt; exit 1; }
  cat $OUT/stamps_fine_$cfg.txt
done
echo ALLOK
