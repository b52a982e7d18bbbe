#!/bin/bash
# wave-kernel bring-up: the new GPU tests first (stop at the first failure), then the whole suite, then C4/C3 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04_wave}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "wave" -x -v --timeout 120 --timeout-method thread > $OUT/pytest_wave.log 2>&1 || { echo WAVE_TESTS_FAILED; tail -40 $OUT/pytest_wave.log; exit 1; }
tail -2 $OUT/pytest_wave.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for CFG in c4 c3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --config $CFG --no-cpu --no-e2e --no-pmc > $OUT/bench_$CFG.json 2> $OUT/bench_$CFG.err || { echo BENCH_FAILED; tail -20 $OUT/bench_$CFG.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_$CFG.json').read().strip().splitlines()[-1]); print('$CFG', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('kernel_ms_per_launch'), d.get('kernel_stats', {}).get('k_analyze_w') if isinstance(d.get('kernel_stats'), dict) else '')"
done
echo ALLOK
