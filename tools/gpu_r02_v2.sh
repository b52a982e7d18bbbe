#!/bin/bash
# r02 v2: PCIe duplex probe (SDMA default vs blit kernels) + C5 bench line with in-run PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02_v2
mkdir -p $OUT
timeout -k 10 120 python -u tools/pcie_probe.py > $OUT/pcie_default.json 2>&1 || { echo PROBE1_FAILED; cat $OUT/pcie_default.json; exit 1; }
HSA_ENABLE_SDMA=0 timeout -k 10 120 python -u tools/pcie_probe.py > $OUT/pcie_nosdma.json 2>&1 || { echo PROBE2_FAILED; cat $OUT/pcie_nosdma.json; exit 1; }
cat $OUT/pcie_*.json
timeout -k 10 600 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu --no-e2e > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo BENCH_FAILED; tail -30 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
echo ALLOK
