#!/bin/bash
# r02 v4: full GPU tests, C5 bench (+ in-run PMC) and C5 phase timing after the 32-bps LDS cut
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02_v4
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 600 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu --no-e2e > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo BENCH_FAILED; tail -30 $OUT/bench_c5.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_c5.json')); r=d['roofline']; print('C5', d['value'], d['ms_per_step'], r['kernel_ms_per_launch'], r['valu_issue_frac'], r['counters'].get('valu_per_wave'))"
for k in 1 8 2 3 5 4; do
  timeout -k 10 200 python -u tools/diag_phases.py flac-raster_amd/flac_raster/_lib/diag/libflac_raster_amd_diag$k.so c5 >> $OUT/c5_phases.txt 2>&1 || { echo DIAG_FAILED; tail $OUT/c5_phases.txt; exit 1; }
done
cat $OUT/c5_phases.txt
echo ALLOK
