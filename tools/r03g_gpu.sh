#!/bin/bash
# round 3: glossy-prior GPU tests, then C3 quality per fraction mode with the prior
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03g
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal status $1 in $2"; exit 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_glossy_prior.py tests/test_gpu_learned_fraction.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1; s=$?; tail -8 $O/tests.log; fatal $s tests
[ $s -eq 0 ] || exit 1
for m in fixed learned albedo; do
  timeout -k 10 300 python -u tools/quality_c3.py --gt tests/golden/c3_gt.npz --props "{\"bsdfSamplingFractionBound\": \"$m\", \"glossyPrior\": true}" > $O/q_$m.log 2>&1 || { s=$?; echo "quality $m failed"; tail -20 $O/q_$m.log; fatal $s q; exit 1; }
  tail -1 $O/q_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['guided_discard']; u=d['unguided_equal_spp']; print('$m+prior', d['guided_vs_unguided'], 'g', g['relmse_exposed'], g['relmse_exposed_trim999'], g['relmse_exposed_dark'], g['seconds'], 'u', u['relmse_exposed'], u['relmse_exposed_trim999'], u['relmse_exposed_dark'], u['seconds'])"
done
