#!/bin/bash
# per-phase counters (k_analyze_w phase-stop builds) + in-kernel phase stamps of the current build, C4
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r05_phases}
STOPLIB=wstop bash tools/pmc_stall_phases.sh $TAG c4 1 2 3 4 5 6 7 full || { echo PHASES_FAILED; exit 1; }
python tools/pmc_stall_table.py gpurun_out/$TAG k_analyze_w > gpurun_out/$TAG/table.txt 2>&1
cat gpurun_out/$TAG/table.txt
timeout -k 10 200 python tools/wstamp_phases.py c4 > gpurun_out/$TAG/wstamps.txt 2>&1 || { echo STAMPS_FAILED; tail gpurun_out/$TAG/wstamps.txt; exit 1; }
cat gpurun_out/$TAG/wstamps.txt
echo ALLOK
