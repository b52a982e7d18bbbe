#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r02_v19b
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1 || { echo PARITY_FAILED; tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
