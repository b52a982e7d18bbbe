#!/bin/bash
# r05: PMC mix (incl. the I-cache / issue pass) of the analysis kernel for one library, then a same-box step.
# usage: bash tools/gpu_r05_pmc.sh <tag> <lib|-> [kernel-filter]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; L=${2:--}; KERN=${3:-k_analyze_w}
[ "$L" != "-" ] && L=$(readlink -f "$L")
LIB=$L bash tools/pmc_mix.sh $TAG || { echo PMC_FAILED; exit 1; }
python tools/pmc_table.py gpurun_out/$TAG $KERN > gpurun_out/$TAG/table.txt 2>&1
cat gpurun_out/$TAG/table.txt; cat gpurun_out/$TAG/fail.log 2>/dev/null
echo ALLOK
