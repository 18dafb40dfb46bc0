#!/bin/bash
# Round 6: k_rays at 7 waves/SIMD (69 VGPRs, no spills) against 8 (64, 7 spilled), with the leaf pairs
set -eo pipefail
OUT=${1:-gpurun_out/r06_rayswaves}
mkdir -p "$OUT"
./tools/ab_multi.sh "$OUT/ab" 3 mitsuba-path-guiding_amd/build/libpgamd.so mitsuba-path-guiding_amd/build_ab/libpgamd.so \
  -- --steps 5 --warmup 1
