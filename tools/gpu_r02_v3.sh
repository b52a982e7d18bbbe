#!/bin/bash
# r02 v3: pipeline tests, e2e variants (H2D-ahead knob), C5 k_analyze phase timing (diag builds)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02_v3
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $OUT/pytest.log; exit 1; }
for A in 0 1 2 3; do
  FRA_H2D_AHEAD=$A timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --steps 5 > $OUT/bench_ahead$A.json 2> $OUT/bench_ahead$A.err || { echo BENCH_FAILED; tail -20 $OUT/bench_ahead$A.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_ahead$A.json')); print('ahead $A', d['value'], json.dumps(d['e2e']))"
done
for k in 1 8 2 3 5 4 6 7; do
  timeout -k 10 200 python -u tools/diag_phases.py flac-raster_amd/flac_raster/_lib/diag/libflac_raster_amd_diag$k.so c5 >> $OUT/c5_phases.txt 2>&1 || { echo DIAG_FAILED; tail $OUT/c5_phases.txt; exit 1; }
done
timeout -k 10 200 python -u tools/diag_phases.py - c5 >> $OUT/c5_phases.txt 2>&1
cat $OUT/c5_phases.txt
echo ALLOK
