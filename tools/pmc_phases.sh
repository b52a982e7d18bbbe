#!/bin/bash
# Per-phase k_analyze instruction counters (run on the GPU box from the repo root):
#   bash tools/pmc_phases.sh <out-subdir>
# needs `make -C flac-raster_amd/csrc diag` built in-tree.  One rocprofv3 PMC pass per
# phase-stop build (no trace domains combined with --pmc).
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
CTRS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY"
for k in 1 2 3 4 5 6 7; do
  timeout -k 10 200 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/d$k -o run -- \
    python $GRAFT_REPO_ROOT/tools/diag_phases.py $GRAFT_REPO_ROOT/flac-raster_amd/flac_raster/_lib/diag/libflac_raster_amd_diag$k.so > $OUT/d$k.log 2>&1
done
timeout -k 10 200 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/full -o run -- \
  python $GRAFT_REPO_ROOT/tools/diag_phases.py - > $OUT/full.log 2>&1
for k in 1 2 3 4 5 6 7; do
  timeout -k 10 100 python $GRAFT_REPO_ROOT/tools/diag_phases.py $GRAFT_REPO_ROOT/flac-raster_amd/flac_raster/_lib/diag/libflac_raster_amd_diag$k.so >> $OUT/times.log 2>&1
done
timeout -k 10 100 python $GRAFT_REPO_ROOT/tools/diag_phases.py - >> $OUT/times.log 2>&1
echo done
