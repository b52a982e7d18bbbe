#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dw_trace
timeout -k 5 200 python -u tools/dw_trace.py > gpurun_out/dw_trace/log.txt 2>&1; echo rc $?
grep -v Warning gpurun_out/dw_trace/log.txt | tail -30
rm -f gpurun_out/dw_trace/trace.bin
