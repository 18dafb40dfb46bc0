#!/bin/bash
# round 5 (w): device logf / double log rounding against math::fastlog over every tracking argument, and
# the C5 GPU/oracle agreement with the reference's fastlog restated on both sides (double libm)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 120 tools/log_rounding > $O/log_rounding.json 2>&1 || exit 1
cat $O/log_rounding.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_volume.py -m gpu -q -rP --timeout 250 --timeout-method thread > $O/vol_tests.log 2>&1; s=$?
grep -E "passed|failed|FAILED|c5 |tracking" $O/vol_tests.log | head -30; [ $s -eq 0 ] || exit 1
