#!/bin/bash
# round 3, first GPU call: GPU suite, the default bench line, and the --gpus 2 launcher (gloo, ranks share the GPU)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03a_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r03a_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03a_gpu_tests.log
timeout -k 10 420 python -u bench.py > gpurun_out/r03a_bench_c3.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r03a_bench_c3.log; exit 1; }
tail -c 3000 gpurun_out/r03a_bench_c3.log
PG_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --quick --no-cpu > gpurun_out/r03a_gloo2_quick.log 2>&1 || { echo "gloo2 failed"; tail -30 gpurun_out/r03a_gloo2_quick.log; exit 1; }
tail -c 1500 gpurun_out/r03a_gloo2_quick.log
