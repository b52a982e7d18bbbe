#!/bin/bash
# Round-3 GPU call (rewritten per call; git history keeps each version).  Usage: bash tools/gpu_r03.sh <tag>
# v19: 7 waves/SIMD (72 VGPRs, 94 SGPRs, no residual keep) with the L2 prefetch (distance 1536 / 1792), and
# prefetch distances 1024 / 2048 for the 6-wave product build, s_setprio 2 on the single-wave phases;
# C4 and C3, alternating, 3 reps.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
D=$GRAFT_REPO_ROOT/flac-raster_amd/flac_raster/_lib/diag
run() {  # lib-or-empty tag cfg
  FRA_LIB_PATH=$1 timeout -k 10 300 python -u bench.py --config $3 --no-cpu --no-e2e --no-pmc --no-trace > $OUT/b.json 2> $OUT/b.err || { echo BENCH_FAILED $2 $3; tail -20 $OUT/b.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-4s %-11s %10.1f MPix/s %8.4f ms/step' % ('$3', '$2', d['value'], d['ms_per_step']), r['kernel_ms_per_launch'])" | tee -a $OUT/ab.txt
}
for rep in 1 2 3; do
  for cfg in c4 c3; do
    run "" prod $cfg; run $D/libflac_raster_amd_exp_w7k0.so w7k0 $cfg; run $D/libflac_raster_amd_exp_w7k0pf1792.so w7k0pf1792 $cfg
    run $D/libflac_raster_amd_exp_pf1024.so pf1024 $cfg; run $D/libflac_raster_amd_exp_pf2048.so pf2048 $cfg
    run $D/libflac_raster_amd_exp_prio2.so prio2 $cfg
  done
done
echo ALLOK
