set -o pipefail
mkdir -p gpurun_out/r02_v0
cd $GRAFT_REPO_ROOT
(rocprofv3 -L > gpurun_out/r02_v0/counters.txt 2>&1 || true)
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r02_v0/pytest_gpu.log 2>&1 && \
timeout -k 10 900 bash tools/profile_config.sh r02_c5_v0 c5 2 && echo ALLOK
