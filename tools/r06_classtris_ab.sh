#!/bin/bash
# Round 6: material-class queue entries carry the hit triangle (PG_CLASS_TRIS) — parity on the new build,
# then A/B against the previous revision (build_ab)
set -eo pipefail
OUT=${1:-gpurun_out/r06_classtris}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_params.py \
  tests/test_gpu_envmap.py tests/test_gpu_xml.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
./tools/ab_bench.sh "$OUT/ab" mitsuba-path-guiding_amd/build_ab/libpgamd.so mitsuba-path-guiding_amd/build/libpgamd.so --steps 5 --warmup 1
