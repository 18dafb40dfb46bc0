#!/bin/bash
# Round 6: one fused BSDF eval + pdf at the NEE and D-tree-sampled directions (bsdfEvalPdf)

set -eo pipefail
OUT=${1:-gpurun_out/r06_evalpdf}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_params.py \
  tests/test_gpu_envmap.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
./tools/ab_bench.sh "$OUT/ab" mitsuba-path-guiding_amd/build_ab/libpgamd.so mitsuba-path-guiding_amd/build/libpgamd.so --steps 5 --warmup 1
