#!/bin/bash
# round 5 (an): path lanes in flight re-measured on the current kernels: 2 / 3 (default) / 4, C3 and C5 x2
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05an
mkdir -p $O
for i in 1 2; do
  for n in 2 3 4; do
    timeout -k 10 240 python bench.py --no-cpu --no-quality --lanes $n > $O/c3_l${n}_$i.log 2>&1 || exit 1
    timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality --lanes $n > $O/c5_l${n}_$i.log 2>&1 || exit 1
  done
done
for f in $O/c*_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
