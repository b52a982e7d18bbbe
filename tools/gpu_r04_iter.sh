#!/bin/bash
# one iteration: wave-kernel GPU tests, C4 bench (serial + pipelined, no counters), per-wave stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04_iter}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_integration.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for CFG in ${CFGS:-c4}; do
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --config $CFG --no-cpu --no-e2e --no-pmc > $OUT/bench_$CFG.json 2> $OUT/bench_$CFG.err || { echo BENCH_FAILED; tail -20 $OUT/bench_$CFG.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_$CFG.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$CFG', d['ms_per_step'], d['config']['serial_ms_per_step'], r['kernel_ms_per_launch'])"
done
if [ "$STAMPS" != 0 ]; then
timeout -k 10 200 python -u tools/wstamp_phases.py c4 > $OUT/wstamps_c4.txt 2>&1 || { echo WSTAMPS_FAILED; tail -20 $OUT/wstamps_c4.txt; exit 1; }
cat $OUT/wstamps_c4.txt
fi
echo ALLOK
