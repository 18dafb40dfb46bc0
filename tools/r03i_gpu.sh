#!/bin/bash
# round 3: guided vs unguided at equal time (best-of-3 clocks) on C3 and on the indirectly lit
# ajar_diffuse variant, per fraction mode
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03i
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal status $1 in $2"; exit 1;; esac; }
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['guided_discard']; u=d['unguided_equal_spp']; e=d['unguided_equal_time']; print('$2', d['guided_vs_unguided'], 'g', g['relmse_exposed'], g['relmse_exposed_trim999'], g['relmse_exposed_dark'], g['seconds'], 'u', u['relmse_exposed'], u['relmse_exposed_trim999'], u['relmse_exposed_dark'], u['seconds'], 'eq', e['relmse_exposed'], e['relmse_exposed_trim999'], e['relmse_exposed_dark'], e['spp'])"; }
timeout -k 10 400 python -u tools/quality_c3.py --scene ajar_diffuse --gt-spp 65536 --save-gt $O/diffuse_gt.npz --props '{"bsdfSamplingFractionBound": "albedo", "glossyPrior": true}' > $O/d_albedo_prior.log 2>&1 || { s=$?; tail -5 $O/d_albedo_prior.log; fatal $s gt; exit 1; }
summ $O/d_albedo_prior.log diffuse-albedo+prior
for cfg in 'fixed|{}' 'learned+prior|{"bsdfSamplingFractionBound": "learned", "glossyPrior": true}'; do
  n=${cfg%%|*}; p=${cfg#*|}
  timeout -k 10 300 python -u tools/quality_c3.py --scene ajar_diffuse --gt $O/diffuse_gt.npz --props "$p" > $O/d_$n.log 2>&1 || { s=$?; tail -5 $O/d_$n.log; fatal $s d; exit 1; }
  summ $O/d_$n.log diffuse-$n
done
for cfg in 'albedo+prior|{"bsdfSamplingFractionBound": "albedo", "glossyPrior": true}' 'learned+prior|{"bsdfSamplingFractionBound": "learned", "glossyPrior": true}'; do
  n=${cfg%%|*}; p=${cfg#*|}
  timeout -k 10 300 python -u tools/quality_c3.py --gt tests/golden/c3_gt.npz --props "$p" > $O/c3_$n.log 2>&1 || { s=$?; tail -5 $O/c3_$n.log; fatal $s c3; exit 1; }
  summ $O/c3_$n.log c3-$n
done
