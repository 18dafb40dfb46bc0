#!/bin/bash
# round 5 (am): small-pass threshold re-measured on the current kernels (PG_SMALL_PASS_PATHS: passes up to this
# many paths run as one chunk; default 2^21): 2^20 / default / 2^22 / 0 (every pass split over the lanes), C3 x2
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05am
mkdir -p $O
for i in 1 2; do
  for t in 1048576 default 4194304 0; do
    if [ $t = default ]; then timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_${t}_$i.log 2>&1 || exit 1
    else PG_SMALL_PASS_PATHS=$t timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_${t}_$i.log 2>&1 || exit 1; fi
  done
done
for f in $O/c*_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d.get('phases', ''))"; done
