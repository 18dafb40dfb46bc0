#!/bin/bash
# Round 6: leaf triangles tested two at a time with both first rows loaded up front (PG_LEAF_PAIRS) — parity on
# the new build, then A/B against PG_LEAF_PAIRS=0 (build_ab)
set -eo pipefail
OUT=${1:-gpurun_out/r06_leafpairs}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_params.py \
  tests/test_gpu_envmap.py tests/test_gpu_xml.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
./tools/ab_bench.sh "$OUT/ab" mitsuba-path-guiding_amd/build_ab/libpgamd.so mitsuba-path-guiding_amd/build/libpgamd.so --steps 5 --warmup 1
