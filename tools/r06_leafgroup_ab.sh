#!/bin/bash
# Round 6: closest-hit leaf triangles per step 2 / 3 / 4 (PG_LEAF_PAIRS) — parity of 4, then a round-robin A/B/C
set -eo pipefail
OUT=${1:-gpurun_out/r06_leafgroup}
mkdir -p "$OUT"
PG_LIB=mitsuba-path-guiding_amd/build_ab3/libpgamd.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_configs.py tests/test_gpu_params.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
./tools/ab_multi.sh "$OUT/ab" 2 mitsuba-path-guiding_amd/build_ab/libpgamd.so mitsuba-path-guiding_amd/build_ab2/libpgamd.so \
  mitsuba-path-guiding_amd/build_ab3/libpgamd.so -- --steps 5 --warmup 1
