#!/bin/bash
# VALU/LDS/SALU instructions per wave of k_analyze up to each diagnostic stop (csrc/Makefile `diag`),
# one rocprofv3 PMC pass per library:  bash tools/pmc_valu_phases.sh <tag> [config] [stops...]
set -e
TAG=$1
CFG=${2:-c4}
shift 2 || true
STOPS=${@:-1 9 8 2 3 5 6 7 4 full}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
for k in $STOPS; do
  if [ $k = full ]; then LIB=-; else LIB=$GRAFT_REPO_ROOT/flac-raster_amd/flac_raster/_lib/diag/libflac_raster_amd_diag$k.so; fi
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES \
    --output-format csv -d $OUT/s$k -o run -- python $GRAFT_REPO_ROOT/tools/diag_phases.py $LIB $CFG > $OUT/s$k.log 2>&1
done
echo done
