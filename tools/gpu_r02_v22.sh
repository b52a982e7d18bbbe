#!/bin/bash
# r02 v22: LIGHT k_assemble (tree tables in global memory, 9.3 KiB LDS) for 32-bps plans: co-resides with
# the 32-bps k_analyze -- parity, then C5 light vs not, and C4 light (A/B on one box)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02_v22}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in 0 1 0 1; do
  FRA_ASM_LIGHT=$v timeout -k 10 300 python -u bench.py --config c5 --no-cpu --no-e2e --no-pmc > $OUT/c5_$v.json 2> $OUT/c5_$v.err || { echo BENCH_FAILED; tail -20 $OUT/c5_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/c5_$v.json').read().strip().splitlines()[-1]); print('c5 light=$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
done
for v in 0 1; do
  FRA_ASM_LIGHT=$v timeout -k 10 200 python -u bench.py --no-cpu --no-e2e --no-pmc > $OUT/c4_$v.json 2> $OUT/c4_$v.err || { echo BENCH_FAILED; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/c4_$v.json').read().strip().splitlines()[-1]); print('c4 light=$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
done
echo ALLOK
