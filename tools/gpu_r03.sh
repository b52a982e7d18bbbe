#!/bin/bash
# Round-3 GPU call (rewritten per call; git history keeps each version).  Usage: bash tools/gpu_r03.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
L=flac-raster_amd/flac_raster/_lib/diag
for v in w7k1 w7k0 w6k0 w5k0 w5lds w5pad500 w5pad1000; do
  timeout -k 10 120 python -u tools/diag_phases.py $L/libflac_raster_amd_exp_$v.so c4 >> $OUT/exp.txt 2>&1 || { echo EXP_FAILED $v; tail $OUT/exp.txt; exit 1; }
done
for lds in 9900 18100; do
  echo "FRA_EXP_LDS=$lds" >> $OUT/exp.txt
  FRA_EXP_LDS=$lds timeout -k 10 120 python -u tools/diag_phases.py $L/libflac_raster_amd_exp_w5lds.so c4 >> $OUT/exp.txt 2>&1 || { echo EXP2_FAILED; tail $OUT/exp.txt; exit 1; }
done
cat $OUT/exp.txt
timeout -k 10 120 python -u tools/stamp_phases.py c4 --fine > $OUT/stamps_c4_fine.txt 2>&1 || { echo STAMP_FAILED; tail -20 $OUT/stamps_c4_fine.txt; exit 1; }
cat $OUT/stamps_c4_fine.txt
timeout -k 10 300 python -u bench.py --config c4 --no-cpu --no-e2e --no-pmc --no-trace > $OUT/c4.json 2> $OUT/c4.err || { echo C4_FAILED; tail -20 $OUT/c4.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/c4.json').read().strip().splitlines()[-1]); print('c4', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
echo ALLOK
