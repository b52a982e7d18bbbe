#!/bin/bash
# Issue / stall breakdown of k_analyze per diagnostic phase stop (csrc/Makefile `diag`): one rocprofv3
# PMC pass per library with 8 SQ counters (WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY,
# quad-cycles; MI355X_MICROARCH.md "rocprofv3 PMC slots").  Post-process: tools/pmc_stall_table.py.
#   bash tools/pmc_stall_phases.sh <out-subdir> [config] [stops...]      (GPU box, repo root)
#   STOPLIB=wstop: the k_analyze_w phase-stop builds (csrc/Makefile `wstops`) instead of k_analyze's `diag`
set -o pipefail
TAG=$1
CFG=${2:-c4}
shift 2 || true
STOPS=${@:-1 9 8 2 3 5 6 7 full}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
for k in $STOPS; do
  if [ $k = full ]; then LIB=-; else LIB=$GRAFT_REPO_ROOT/flac-raster_amd/flac_raster/_lib/diag/libflac_raster_amd_${STOPLIB:-diag}$k.so; fi
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    --output-format csv -d $OUT/a$k -o run -- python $GRAFT_REPO_ROOT/tools/diag_phases.py $LIB $CFG > $OUT/a$k.log 2>&1 \
    || { echo "pass a$k failed"; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT \
    SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_BUSY_CYCLES \
    --output-format csv -d $OUT/b$k -o run -- python $GRAFT_REPO_ROOT/tools/diag_phases.py $LIB $CFG > $OUT/b$k.log 2>&1 \
    || { echo "pass b$k failed"; exit 1; }
done
echo done
