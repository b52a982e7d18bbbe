#!/bin/bash
# Round-3 GPU call (rewritten per call; git history keeps each version).  Usage: bash tools/gpu_r03.sh <tag>
# v9: final pipelined-assembly defaults (16-bit: k_assemble, 32-bps: k_assemble_bg; frame-size chain on the
# pack stream) -- full GPU suite, A/B against FRA_CHAIN_BG=0 (the r02 arrangement) and FRA_PIPE_ASM forced,
# then a rocprofv3 kernel trace of the pipelined C4 / C5 steps for the timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|error" $OUT/pytest.log | head -20; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
run() {  # asm chain cfg
  FRA_PIPE_ASM=$1 FRA_CHAIN_BG=$2 timeout -k 10 300 python -u bench.py --config $3 --no-cpu --no-e2e --no-pmc --no-trace > $OUT/b.json 2> $OUT/b.err || { echo BENCH_FAILED $1 $2 $3; tail -20 $OUT/b.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); r=d['roofline']; print('%-4s asm=%s chain=%s %10.1f MPix/s %8.4f ms/step' % ('$3', '$1', '$2', d['value'], d['ms_per_step']), r['kernel_ms_per_launch'])" | tee -a $OUT/ab.txt
}
for rep in 1 2 3; do
  for cfg in c4 c3; do
    run -1 1 $cfg; run -1 0 $cfg
  done
done
run -1 1 c5; run 0 1 c5; run -1 0 c5
cd /tmp && export TMPDIR=/tmp
for cfg in c4 c5; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$cfg -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $cfg --steps 12 --warmup 2 --no-cpu --no-e2e --no-pmc --no-trace > $OUT/trace_$cfg.log 2>&1 || { echo TRACE_FAILED $cfg; tail $OUT/trace_$cfg.log; exit 1; }
done
echo ALLOK
