#!/bin/bash
# Round 6: persistent closest-hit lanes (PG_TRACE_PERSIST) — parity on the default build, then A/B against
# the grid-stride rows (build_ab: -DPG_TRACE_PERSIST=0) and a 6-wave variant (build_ab2: -DPG_RAYS_WAVES=6)
set -eo pipefail
OUT=${1:-gpurun_out/r06_persist}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_params.py \
  -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
./tools/ab_bench.sh "$OUT/ab_persist" mitsuba-path-guiding_amd/build_ab/libpgamd.so mitsuba-path-guiding_amd/build/libpgamd.so --steps 5 --warmup 1
./tools/ab_bench.sh "$OUT/ab_waves6" mitsuba-path-guiding_amd/build_ab/libpgamd.so mitsuba-path-guiding_amd/build_ab2/libpgamd.so --steps 5 --warmup 1
