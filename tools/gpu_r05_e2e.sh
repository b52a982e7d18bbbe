set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05_d2hw; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread -k "ring or host" > $OUT/pytest.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for C in c3 c4; do
timeout -k 10 600 python3 bench.py --gpus 1 --steps 10 --warmup 3 --config $C --no-cpu --no-pmc --no-trace > $OUT/bench_$C.json 2> $OUT/bench_$C.err || { echo BENCH_FAILED $C; tail -20 $OUT/bench_$C.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['e2e']; print(sys.argv[1], e['ms'], e.get('pageable'), {k: (v['ms'], v['decode_ms']) for k, v in e['e2e_file'].items() if isinstance(v, dict)})" $OUT/bench_$C.json
done
timeout -k 10 900 python3 bench.py --gpus 1 --steps 3 --warmup 2 --config c5 --no-cpu --no-pmc --no-trace > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo BENCH_FAILED c5; tail -20 $OUT/bench_c5.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(json.dumps(d['e2e']))" $OUT/bench_c5.json
echo ALLOK
