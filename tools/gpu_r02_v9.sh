#!/bin/bash
# r02 v9: cross-execute pipelining (double-buffered slots, k_assemble on its own stream): GPU tests, A/B on C3/C4/C5
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02_v9
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for C in c4 c3 c5; do for P in 0 1; do
  ST=20; [ $C = c5 ] && ST=5
  FRA_PIPE=$P timeout -k 10 400 python -u bench.py --config $C --steps $ST --warmup 2 --no-cpu --no-e2e --no-pmc > $OUT/bench_${C}_p$P.json 2> $OUT/bench_${C}_p$P.err || { echo BENCH_FAILED; tail -30 $OUT/bench_${C}_p$P.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_${C}_p$P.json')); print('$C pipe=$P', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'], d['pyflac_shim_c2'])"
done; done
echo ALLOK
