#!/bin/bash
# PMC mix of the analysis kernels (current build) -> table
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r04_pmc}
bash tools/pmc_mix.sh $TAG || { echo PMC_FAILED; exit 1; }
python tools/pmc_table.py gpurun_out/$TAG ${KERN:-k_analyze_w} > gpurun_out/$TAG/table.txt 2>&1; cat gpurun_out/$TAG/table.txt; cat gpurun_out/$TAG/fail.log 2>/dev/null
echo ALLOK
