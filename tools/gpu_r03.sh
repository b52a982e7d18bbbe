#!/bin/bash
# Round-3 GPU call (rewritten per call; git history keeps each version).  Usage: bash tools/gpu_r03.sh <tag>
# v21: defaults now k_assemble4 (a frame per wave) and, for 32-bps pipelined plans, k_assemble_bg with a
# frame per wave -- full GPU suite, then C5 A/B of the background form per wave vs per workgroup (x2),
# C4 / C3 sanity.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
D=$GRAFT_REPO_ROOT/flac-raster_amd/flac_raster/_lib/diag
run() {  # lib tag cfg
  FRA_LIB_PATH=$1 timeout -k 10 300 python -u bench.py --config $3 --no-cpu --no-e2e --no-pmc --no-trace > $OUT/b.json 2> $OUT/b.err || { echo BENCH_FAILED $2 $3; tail -20 $OUT/b.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-4s %-6s %10.1f MPix/s %8.4f ms/step' % ('$3', '$2', d['value'], d['ms_per_step']), r['kernel_ms_per_launch'])" | tee -a $OUT/ab.txt
}
for rep in 1 2; do
  run "" bgwave c5; run $D/libflac_raster_amd_exp_bgwg.so bgwg c5
done
run "" prod c4; run "" prod c3
echo ALLOK
