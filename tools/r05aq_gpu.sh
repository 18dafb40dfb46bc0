#!/bin/bash
# round 5 (aq): the deep-S-tree lookup test (descent below the jump grid) and the full GPU suite
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05aq
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rP --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?
grep -E "passed|failed|FAILED|deep" $O/gpu_tests.log | head -20; exit $s
