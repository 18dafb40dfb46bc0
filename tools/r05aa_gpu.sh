#!/bin/bash
# round 5 (aa): GPU suite at the fastlog / contraction commit with the tightened C5 bars and the unit-level
# parity prints (BSDF, HG, lookups) used to tighten the remaining bars
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rP --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?
grep -E "passed|failed|FAILED|c3 |c4 |c5 |tracking|bsdf |hg:|lookups:" $O/gpu_tests.log | head -40; exit $s
