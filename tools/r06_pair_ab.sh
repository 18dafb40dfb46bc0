#!/bin/bash
# Round 6: two closest-hit walks per lane (PG_TRACE_PAIR) — parity on the paired build (build_ab: 4 waves/SIMD),
# then A/B against the default build; build_ab2: 5 waves/SIMD (spills)
set -eo pipefail
OUT=${1:-gpurun_out/r06_pair}
mkdir -p "$OUT"
PG_LIB=mitsuba-path-guiding_amd/build_ab/libpgamd.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_configs.py tests/test_gpu_params.py tests/test_gpu_envmap.py tests/test_gpu_xml.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
./tools/ab_bench.sh "$OUT/ab_pair4" mitsuba-path-guiding_amd/build/libpgamd.so mitsuba-path-guiding_amd/build_ab/libpgamd.so --steps 5 --warmup 1
./tools/ab_bench.sh "$OUT/ab_pair5" mitsuba-path-guiding_amd/build/libpgamd.so mitsuba-path-guiding_amd/build_ab2/libpgamd.so --steps 5 --warmup 1
