#!/bin/bash
# round 3 end: GPU suite and smoke() at HEAD
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03zp
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?; tail -3 $O/gpu_tests.log; [ $s -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
