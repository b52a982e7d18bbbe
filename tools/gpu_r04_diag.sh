#!/bin/bash
# diagnostics of the analysis: per-wave phase stamps (k_analyze_w) + a bench line with in-run counters
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04_diag}
CFG=${2:-c4}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/wstamp_phases.py $CFG > $OUT/wstamps_$CFG.txt 2>&1 || { echo WSTAMPS_FAILED; tail -20 $OUT/wstamps_$CFG.txt; exit 1; }
cat $OUT/wstamps_$CFG.txt
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --config $CFG --no-cpu --no-e2e > $OUT/bench_$CFG.json 2> $OUT/bench_$CFG.err || { echo BENCH_FAILED; tail -20 $OUT/bench_$CFG.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_$CFG.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], r['kernel_ms_per_launch']); print(json.dumps(r['counters']))"
echo ALLOK
