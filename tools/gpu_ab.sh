#!/bin/bash
# A/B of two library builds on one box (alternating runs): bash tools/gpu_ab.sh <libA> <libB> [config] [reps]
set -o pipefail
cd $GRAFT_REPO_ROOT
A=$1; B=$2; CFG=${3:-c4}; R=${4:-3}
for i in $(seq $R); do
  timeout -k 10 200 python -u tools/diag_phases.py $A $CFG || exit 1
  timeout -k 10 200 python -u tools/diag_phases.py $B $CFG || exit 1
done
