#!/bin/bash
# Round-3 GPU call (rewritten per call; git history keeps each version).  Usage: bash tools/gpu_r03.sh <tag>
# v27: A/B of the k_analyze prologue candidate (normalisation parameters read only off the LUT fast path;
# built as the experiment library pro1 from DESIGN §9's candidate) against the product build, C4 / C3
# (3 alternating reps); pipeline + parity tests on the candidate first.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
B1=$GRAFT_REPO_ROOT/flac-raster_amd/flac_raster/_lib/diag/libflac_raster_amd_exp_pro1.so
FRA_LIB_PATH=$B1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_pro1.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/pytest_pro1.log; exit 1; }
tail -1 $OUT/pytest_pro1.log
run() {  # candidate(1)/product(0) cfg
  if [ "$1" = 1 ]; then export FRA_LIB_PATH=$B1; else unset FRA_LIB_PATH; fi
  timeout -k 10 300 python -u bench.py --config $2 --no-cpu --no-e2e --no-pmc --no-trace > $OUT/b.json 2> $OUT/b.err || { echo BENCH_FAILED $1 $2; tail -20 $OUT/b.err; exit 1; }
  unset FRA_LIB_PATH
  python -c "import json,sys; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-4s cand=%s %10.1f MPix/s %9.4f ms/step' % ('$2', '$1', d['value'], d['ms_per_step']), r['kernel_ms_per_launch'])" | tee -a $OUT/ab.txt
}
for rep in 1 2 3; do
  for cfg in c4 c3; do run 1 $cfg; run 0 $cfg; done
done
echo ALLOK
