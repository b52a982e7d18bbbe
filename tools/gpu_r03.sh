#!/bin/bash
# Round-3 GPU call (rewritten per call; git history keeps each version).  Usage: bash tools/gpu_r03.sh <tag>
# v26: the frame-size chain of small frame groups as ONE single-workgroup launch (k_frame_chain1, groups of
# <= 4096 frames; FRA_CHAIN1=0 = the k_frame_bytes + device scan + k_group_offsets chain) -- full GPU suite
# on it, then A/B on the default C4 line (HBM step, pyflac shim per-stream time, e2e host-band pipeline)
# and on the 8-way C4 / C3 shares, 3 alternating reps each.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; grep -E "FAIL|Error|error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
FRA_CHAIN1=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_host.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_chain0.log 2>&1 || { echo TESTS0_FAILED; tail -30 $OUT/pytest_chain0.log; exit 1; }
tail -1 $OUT/pytest_chain0.log
full() {  # chain1_max
  FRA_CHAIN1=$1 timeout -k 10 400 python -u bench.py --no-cpu --no-pmc --no-trace > $OUT/b.json 2> $OUT/b.err || { echo BENCH_FAILED $1; tail -20 $OUT/b.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('c4 chain1=%-5s %9.1f MPix/s %7.4f ms  shim %.3f ms/stream  e2e %.2f ms' % ('$1', d['value'], d['ms_per_step'], d['pyflac_shim_c2']['ms_per_stream'], d['e2e']['ms']), d['roofline']['kernel_ms_per_launch'])" | tee -a $OUT/ab.txt
}
shard() {  # chain1_max cfg r/N
  FRA_CHAIN1=$1 timeout -k 10 300 python -u bench.py --config $2 --shard $3 --no-cpu --no-e2e --no-pmc --no-trace > $OUT/b.json 2> $OUT/b.err || { echo SHARD_FAILED $1 $2; tail -20 $OUT/b.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('%s %s chain1=%-5s %8.4f ms/step' % ('$2', '$3', '$1', d['ms_per_step']), d['kernel_ms_per_launch'])" | tee -a $OUT/ab.txt
}
for rep in 1 2 3; do full 4096; full 0; done
for rep in 1 2 3; do shard 4096 c4 4/8; shard 0 c4 4/8; shard 4096 c3 0/8; shard 0 c3 0/8; done
echo ALLOK
