#!/bin/bash
# r06 GPU session steps, each under its own time limit, stopping at the first GPU step that crashes / times out.
# usage: bash tools/gpu_r06.sh <tag> <step> [<step> ...]
#   tests           pytest -m gpu (all)
#   bench:<cfg>     bench.py --config <cfg> (default steps, counters, trace) -> bench_<cfg>.json
#   mmfetch:<lib>   FETCH_SIZE + WRITE_SIZE passes of the C4 plan's kernels (bench --child) with library <lib>
#   list            rocprofv3 -L (the counters of this box)
#   ab:<cfg>:<lib>[:ENV=V,...]  tools/ab_step.py (same-box pipelined step)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for S in "$@"; do
  echo "== $S $(date +%T)"
  case $S in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread ${TESTK:+-k "$TESTK"} > $OUT/pytest.log 2>&1
      rc=$?; tail -5 $OUT/pytest.log; grep -E "FAILED|ERROR" $OUT/pytest.log | head -20
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS_ABORTED rc=$rc"; exit 1; fi ;;
    bench:*)
      C=${S#bench:}
      timeout -k 10 500 python -u bench.py --config $C ${BENCHARGS} --prof-dir $OUT/prof > $OUT/bench_$C.json 2> $OUT/bench_$C.err || { echo "BENCH_FAILED $C"; tail -20 $OUT/bench_$C.err; exit 1; }
      python - $OUT/bench_$C.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=d["roofline"]; c=r.get("counters") or {}
print(d["value"], d["ms_per_step"], r["kernel_ms_per_launch"], r["frac"], c.get("traffic_by_kernel"), c.get("valu_per_wave"), c.get("stalls"), d.get("analysis_instance"))
print((d.get("kernel_stats") or {}).get("kernels"))
PY
      ;;
    mmfetch:*)
      L=${S#mmfetch:}; N=$(basename $L .so)
      for CT in FETCH_SIZE WRITE_SIZE; do
        cd /tmp
        FRA_LIB_PATH=$GRAFT_REPO_ROOT/$L timeout -s KILL 120 rocprofv3 --pmc $CT --output-format csv -d $OUT/mm_${N}_$CT -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config ${MMCFG:-c4} --steps 1 --warmup 1 --child > $OUT/mm_${N}_$CT.log 2>&1 || { echo "PMC_FAILED $N $CT"; exit 1; }
        cd $GRAFT_REPO_ROOT
      done
      python tools/pmc_kernel_table.py $OUT/mm_${N}_FETCH_SIZE $OUT/mm_${N}_WRITE_SIZE ;;
    list)
      cd /tmp; timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1; cd $GRAFT_REPO_ROOT; grep -c . $OUT/counters.txt ;;
    ab:*)
      IFS=: read -r _ C L E <<< "$S"
      timeout -k 10 200 python -u tools/ab_step.py $C $L ${E//,/ } >> $OUT/ab.txt 2>&1 || { echo "AB_FAILED $S"; tail -20 $OUT/ab.txt; exit 1; }
      tail -1 $OUT/ab.txt ;;
  esac
done
echo ALLOK
