#!/bin/bash
# Round 6: triangle records in blocks of 8 (PG_TRI_BLOCKED, first rows in one line) — parity on the new build,
# then A/B/C: three consecutive rows per triangle (build_ab: PG_TRI_BLOCKED=0), blocked (build), blocked with
# the 8-wide BVH's 80-B nodes padded to 128 B (build_ab2: PG_WIDE_NODE_F4=8)
set -eo pipefail
OUT=${1:-gpurun_out/r06_triblock}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_params.py \
  -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
./tools/ab_multi.sh "$OUT/ab" 2 mitsuba-path-guiding_amd/build_ab/libpgamd.so mitsuba-path-guiding_amd/build/libpgamd.so \
  mitsuba-path-guiding_amd/build_ab2/libpgamd.so -- --steps 5 --warmup 1
