#!/bin/bash
# round 4: the volumetric tile-shard test, then the whole GPU suite
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_volume.py -x -v --timeout 250 --timeout-method thread -k tile_shard > $O/shard.log 2>&1; s=$?; tail -4 $O/shard.log; [ $s -eq 0 ] || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?; grep -E "passed|failed|FAILED" $O/gpu_tests.log | head; [ $s -eq 0 ] || exit 1
