#!/bin/bash
# Round 6: material records loaded once per distinct material of the wave at a uniform address (PG_MAT_UNIFORM=1, build_ab) —
# parity on that build, then A/B against the per-lane gather
set -eo pipefail
OUT=${1:-gpurun_out/r06_matuniform}
mkdir -p "$OUT"
PG_LIB=mitsuba-path-guiding_amd/build_ab/libpgamd.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_configs.py tests/test_gpu_params.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
./tools/ab_bench.sh "$OUT/ab" mitsuba-path-guiding_amd/build/libpgamd.so mitsuba-path-guiding_amd/build_ab/libpgamd.so --steps 5 --warmup 1
