#!/bin/bash
# r02 v18: direct write (k_analyze places subframes, CRC-16, offsets) -- DW tests first, suite, A/B bench
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02_v18}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct_write.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_dw.log 2>&1 || { echo DW_TESTS_FAILED; tail -60 $OUT/pytest_dw.log; exit 1; }
tail -2 $OUT/pytest_dw.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-e2e --no-pmc > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { echo BENCH_FAILED; tail -30 $OUT/bench_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
done
FRA_DW=0 timeout -k 10 200 python -u bench.py --no-cpu --no-e2e --no-pmc > $OUT/bench_nodw.json 2> $OUT/bench_nodw.err || { echo BENCH_FAILED; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_nodw.json').read().strip().splitlines()[-1]); print('nodw', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --no-cpu --no-e2e --no-pmc --steps 20 --warmup 3 > $OUT/stats.log 2>&1 || { echo STATS_FAILED; tail -20 $OUT/stats.log; exit 1; }
echo ALLOK
