#!/bin/bash
# r02 v14: smoke(), 2-rank strong-scaling rehearsal on one GPU (gloo), default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02_v14
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
FRA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 > $OUT/bench_n2.json 2> $OUT/bench_n2.err || { echo N2_FAILED; tail -30 $OUT/bench_n2.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_n2.json').read().strip().splitlines()[-1]); print('N2', d['value'], d['ms_per_step'], d['scaling'], d['per_rank'], d['imbalance'])"
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo ALLOK
