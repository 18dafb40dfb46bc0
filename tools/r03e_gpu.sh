#!/bin/bash
# round 3: C3 quality per fraction mode, then the GPU suite.  Any timeout / abort / segfault ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03e
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal status $1 in $2"; exit 1;; esac; }
for m in learned albedo fixed; do
  timeout -k 10 300 python -u tools/quality_c3.py --gt tests/golden/c3_gt.npz --props "{\"bsdfSamplingFractionBound\": \"$m\"}" > $O/q_$m.log 2>&1 || { s=$?; echo "quality $m failed"; tail -20 $O/q_$m.log; fatal $s q; exit 1; }
  tail -1 $O/q_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['guided_vs_unguided'], d['guided_discard']['relmse_exposed'], d['guided_discard']['relmse_exposed_trim999'], d['unguided_equal_spp']['relmse_exposed'], d['guided_discard']['seconds'])"
done
timeout -k 10 540 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; tail -8 $O/gpu_tests.log
