#!/bin/bash
# Round-3 GPU call (rewritten per call; git history keeps each version).  Usage: bash tools/gpu_r03.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
L=flac-raster_amd/flac_raster/_lib/diag
for rep in 1 2; do
for v in w7k0 w6k1 w6k0 w5k1; do
  timeout -k 10 120 python -u tools/diag_phases.py $L/libflac_raster_amd_exp_$v.so c4 >> $OUT/exp.txt 2>&1 || { echo EXP_FAILED $v; tail $OUT/exp.txt; exit 1; }
done
done
cat $OUT/exp.txt
for cfg in c4 c3; do
timeout -k 10 300 python -u bench.py --config $cfg --no-cpu --no-e2e --no-pmc --no-trace > $OUT/$cfg.json 2> $OUT/$cfg.err || { echo BENCH_FAILED; tail -20 $OUT/$cfg.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/$cfg.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
done
echo ALLOK
