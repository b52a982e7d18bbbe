#!/bin/bash
# same-box A/B of library builds (alternating runs of tools/diag_phases.py): bash tools/gpu_r04_ab.sh <tag> <cfg> <lib>...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; CFG=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2 3; do
  for L in "$@"; do
    timeout -k 10 200 python -u tools/diag_phases.py $L $CFG >> $OUT/ab.txt 2>&1 || { echo AB_FAILED $L; tail -20 $OUT/ab.txt; exit 1; }
  done
done
cat $OUT/ab.txt
echo ALLOK
