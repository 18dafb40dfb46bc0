#!/bin/bash
# Round 6: camera-ray kernel occupancy (PG_TRACE_WAVES): compiler's 6 waves/SIMD against 7 and 8, round-robin
set -eo pipefail
OUT=${1:-gpurun_out/r06_tracewaves}
mkdir -p "$OUT"
./tools/ab_multi.sh "$OUT/ab" 2 mitsuba-path-guiding_amd/build/libpgamd.so mitsuba-path-guiding_amd/build_ab/libpgamd.so \
  mitsuba-path-guiding_amd/build_ab2/libpgamd.so -- --steps 5 --warmup 1
