#!/bin/bash
# round 3: guided vertices only up to depth D (PG_GUIDE_MAX_DEPTH, A/B knob): C3 quality and time
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03v
mkdir -p $O
for dmax in 0 2 3 4; do
  PG_GUIDE_MAX_DEPTH=$dmax timeout -k 10 300 python -u tools/quality_c3.py --gt tests/golden/c3_gt.npz --props '{"bsdfSamplingFractionBound": "albedo", "glossyPrior": true}' > $O/q_d$dmax.log 2>&1 || { tail -5 $O/q_d$dmax.log; exit 1; }
  tail -1 $O/q_d$dmax.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['guided_discard']; u=d['unguided_equal_spp']; print('depth<= $dmax', d['guided_vs_unguided'], 'g', g['relmse_exposed'], g['relmse_exposed_dark'], g['seconds'], g['gsegments_s'], 'u', u['relmse_exposed'], u['relmse_exposed_dark'], u['seconds'], u['gsegments_s'])"
done
