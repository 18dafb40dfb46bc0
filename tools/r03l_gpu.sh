#!/bin/bash
# round 3: C3 guided quality vs training length (albedo + glossy prior), equal spp / equal time
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03l
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal status $1 in $2"; exit 1;; esac; }
for tr in 6 7 8; do
  timeout -k 10 300 python -u tools/quality_c3.py --gt tests/golden/c3_gt.npz --train $tr --props '{"bsdfSamplingFractionBound": "albedo", "glossyPrior": true}' > $O/c3_t$tr.log 2>&1 || { s=$?; tail -5 $O/c3_t$tr.log; fatal $s q; exit 1; }
  tail -1 $O/c3_t$tr.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['guided_discard']; u=d['unguided_equal_spp']; e=d['unguided_equal_time']; print('train $tr', d['guided_vs_unguided'], d['inversevar_vs_unguided'], 'g', g['relmse_exposed'], g['relmse_exposed_trim999'], g['relmse_exposed_dark'], g['seconds'], 'u', u['relmse_exposed'], u['seconds'], 'eq', e['relmse_exposed'], e['spp'])"
done
for tr in 7; do
  timeout -k 10 300 python -u tools/quality_c3.py --scene ajar_diffuse --gt tests/golden/ajar_diffuse_gt.npz --train $tr --props '{"bsdfSamplingFractionBound": "albedo", "glossyPrior": true}' > $O/d_t$tr.log 2>&1 || { s=$?; tail -5 $O/d_t$tr.log; fatal $s q; exit 1; }
  tail -1 $O/d_t$tr.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['guided_discard']; u=d['unguided_equal_spp']; e=d['unguided_equal_time']; print('diffuse train $tr', d['guided_vs_unguided'], d['inversevar_vs_unguided'], 'g', g['relmse_exposed'], g['relmse_exposed_trim999'], g['relmse_exposed_dark'], g['seconds'], 'u', u['relmse_exposed'], u['seconds'], 'eq', e['relmse_exposed'], e['spp'])"
done
