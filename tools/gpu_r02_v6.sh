#!/bin/bash
# r02 v5: grouped LD + 32-bit FIXED sums for 32-bps: full GPU tests, C4/C5 lines, C5 phase timing + PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02_v6
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for C in c5 c4 c3; do
timeout -k 10 600 python -u bench.py --config $C --steps 5 --warmup 1 --no-cpu --no-e2e --no-pmc > $OUT/bench_$C.json 2> $OUT/bench_$C.err || { echo BENCH_FAILED; tail -30 $OUT/bench_$C.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_$C.json')); r=d['roofline']; print('$C', d['value'], d['ms_per_step'], r['kernel_ms_per_launch'])"
done
for k in 1 8 2 3 5 4; do
  timeout -k 10 200 python -u tools/diag_phases.py flac-raster_amd/flac_raster/_lib/diag/libflac_raster_amd_diag$k.so c5 >> $OUT/c5_phases.txt 2>&1 || { echo DIAG_FAILED; tail $OUT/c5_phases.txt; exit 1; }
done
cat $OUT/c5_phases.txt
bash tools/pmc_valu_phases.sh r02_v6/pmc c5 1 8 2 3 5 4 full > /dev/null 2>&1 || echo PMC_PHASES_FAILED
python tools/pmc_phase_table.py $OUT/pmc
echo ALLOK
