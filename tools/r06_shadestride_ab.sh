#!/bin/bash
# Round 6: BVH-order shading records padded from 80 B to one 128-B line (PG_TRI_SHADE_STRIDE=8, build_ab3) —
# parity on that build, then A/B against the default 80-B stride
set -eo pipefail
OUT=${1:-gpurun_out/r06_shadestride}
mkdir -p "$OUT"
PG_LIB=mitsuba-path-guiding_amd/build_ab3/libpgamd.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_configs.py tests/test_gpu_params.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
./tools/ab_bench.sh "$OUT/ab" mitsuba-path-guiding_amd/build/libpgamd.so mitsuba-path-guiding_amd/build_ab3/libpgamd.so --steps 5 --warmup 1
