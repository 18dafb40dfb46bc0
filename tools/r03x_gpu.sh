#!/bin/bash
# round 3: small training passes split over the lanes (PG_SMALL_PASS_PATHS=0) vs one chunk; C3 bench with the CPU ground truth
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03x
mkdir -p $O
for sp in 2097152 0 262144; do
  for w in 8 1; do
    PG_SMALL_PASS_PATHS=$sp PG_TRAIN_ONLY=1 PG_TRAIN_REPS=3 timeout -k 10 200 python -u tools/train_timing.py $w > $O/train_w${w}_sp$sp.log 2>&1 || exit 1
    echo "W=$w small=$sp"; grep "rep 2" $O/train_w${w}_sp$sp.log | cut -c1-60
  done
done
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 1; }
grep "^{" $O/bench_c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['rmse_vs_cpu']))"
