#!/bin/bash
# same-box A/B of pipelined steps (tools/ab_step.py): bash tools/gpu_r04_abs.sh <tag> <cfg> "<lib> [ENV=V ...]" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; CFG=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2 3; do
  for V in "$@"; do
    timeout -k 10 200 python -u tools/ab_step.py $CFG $V >> $OUT/ab.txt 2>&1 || { echo AB_FAILED $V; tail -20 $OUT/ab.txt; exit 1; }
  done
done
cat $OUT/ab.txt
echo ALLOK
