#!/bin/bash
# Round-3 GPU call (rewritten per call; git history keeps each version).  Usage: bash tools/gpu_r03.sh <tag>
# v20: frame assembly with one frame per wave, four per workgroup (k_assemble4, FRA_ASM_WAVE=1: U=2,
# 2: U=4) -- parity of both forms (pipeline + parity tests under the env), then A/B against k_assemble on
# C4 and C3 (3 reps); product build now with the prefetch distance 1024.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for w in 1 2; do
FRA_ASM_WAVE=$w timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_w$w.log 2>&1 || { echo TESTS_FAILED w$w; grep -E "FAIL|Error|error" $OUT/pytest_w$w.log | head; tail -30 $OUT/pytest_w$w.log; exit 1; }
tail -1 $OUT/pytest_w$w.log
done
run() {  # wave cfg
  FRA_ASM_WAVE=$1 timeout -k 10 300 python -u bench.py --config $2 --no-cpu --no-e2e --no-pmc --no-trace > $OUT/b.json 2> $OUT/b.err || { echo BENCH_FAILED $1 $2; tail -20 $OUT/b.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-4s wave=%s %10.1f MPix/s %8.4f ms/step' % ('$2', '$1', d['value'], d['ms_per_step']), r['kernel_ms_per_launch'])" | tee -a $OUT/ab.txt
}
for rep in 1 2 3; do
  for cfg in c4 c3; do
    run 0 $cfg; run 1 $cfg; run 2 $cfg
  done
done
echo ALLOK
