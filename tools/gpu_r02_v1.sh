#!/bin/bash
# r02 v1: GPU tests (incl. the pipelined host path), default bench line (C4), kernel stats of C4
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02_v1
mkdir -p $OUT
(rocprofv3 -L > $OUT/counters.txt 2>&1 || true)
timeout -k 10 400 python -u -m pytest ${PYTEST_SEL:-tests} -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; tail -30 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo ALLOK
