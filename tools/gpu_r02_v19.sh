#!/bin/bash
# r02 v19: direct write opt-in (FRA_DW=1) -- DW tests, full suite, bench (slot default vs FRA_DW=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02_v19}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct_write.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_dw.log 2>&1 || { echo DW_TESTS_FAILED; tail -60 $OUT/pytest_dw.log; exit 1; }
tail -1 $OUT/pytest_dw.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python -u bench.py --no-cpu --no-e2e --no-pmc > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
FRA_DW=1 timeout -k 10 200 python -u bench.py --no-cpu --no-e2e --no-pmc > $OUT/bench_dw.json 2> $OUT/bench_dw.err || { echo BENCH_FAILED; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_dw.json').read().strip().splitlines()[-1]); print('dw', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"

FRA_ASM_WG=4 timeout -k 10 200 python -u bench.py --no-cpu --no-e2e --no-pmc > $OUT/bench_asm4.json 2> $OUT/bench_asm4.err || { echo BENCH_FAILED; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_asm4.json').read().strip().splitlines()[-1]); print('asm4', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
echo ALLOK
