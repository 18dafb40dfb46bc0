#!/bin/bash
# round 3: GPU suite with the learned BSDF-sampling fraction, then C3 quality per fraction mode
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r03c
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03c/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r03c/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03c/gpu_tests.log
for m in learned albedo fixed; do
  timeout -k 10 300 python -u tools/quality_c3.py --gt tests/golden/c3_gt.npz --props "{\"bsdfSamplingFractionBound\": \"$m\"}" > gpurun_out/r03c/q_$m.log 2>&1 || { echo "quality $m failed"; tail -20 gpurun_out/r03c/q_$m.log; exit 1; }
  tail -1 gpurun_out/r03c/q_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['guided_vs_unguided'], d['guided_discard']['relmse_exposed'], d['guided_discard']['relmse_exposed_trim999'], d['unguided_equal_spp']['relmse_exposed'])"
done
