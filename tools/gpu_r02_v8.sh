#!/bin/bash
# r02 v8: GPU tests after the first-frame ABI + incremental pyflac shim; quick C4 line with the shim latency
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02_v8
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu --no-pmc > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['pyflac_shim_c2'], d['e2e']['ms'])"
echo ALLOK
