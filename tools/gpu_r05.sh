#!/bin/bash
# r05 GPU session: [pytest -m gpu] -> same-box A/B of pipelined steps -> [PMC mix of named libraries]
# usage: TESTS=1 PMC="tagA:libA tagB:libB" bash tools/gpu_r05.sh <tag> <cfg> "<lib> [ENV=V ...]" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; CFG=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread ${TESTK:+-k "$TESTK"} > $OUT/pytest.log 2>&1
  rc=$?
  tail -30 $OUT/pytest.log
  # a test failure is reported and the A/B still runs; a crash / timeout of the GPU step ends the call
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo TESTS_ABORTED rc=$rc; exit 1; fi
fi
for r in $(seq ${REPS:-3}); do
  for V in "$@"; do
    timeout -k 10 200 python -u tools/ab_step.py $CFG $V >> $OUT/ab.txt 2>&1 || { echo AB_FAILED $V; tail -20 $OUT/ab.txt; exit 1; }
  done
done
cat $OUT/ab.txt
for P in $PMC; do
  bash tools/gpu_r05_pmc.sh ${TAG}_pmc_${P%%:*} ${P#*:} > $OUT/pmc_${P%%:*}.log 2>&1 || { echo PMC_FAILED $P; exit 1; }
  cat gpurun_out/${TAG}_pmc_${P%%:*}/table.txt
done
echo ALLOK
