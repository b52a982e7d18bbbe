#!/bin/bash
# r02 v10: mid-side stereo (FRA-1 3.1b) GPU parity + regression check of the C4/C3 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02_v10
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for C in c4 c3; do
timeout -k 10 300 python -u bench.py --config $C --no-cpu --no-e2e --no-pmc > $OUT/bench_$C.json 2> $OUT/bench_$C.err || { echo BENCH_FAILED; tail -30 $OUT/bench_$C.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_$C.json')); print('$C', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
done
echo ALLOK
