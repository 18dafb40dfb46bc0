#!/bin/bash
# round 5 (ao): hardware queues per process (GPU_MAX_HW_QUEUES, 4 on the box) against lanes: 3 and 4 lanes at
# 4 and 8 queues, C3 and C5 x2
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05ao
mkdir -p $O
for i in 1 2; do
  for q in 4 8; do
    for n in 3 4; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python bench.py --no-cpu --no-quality --lanes $n > $O/c3_q${q}_l${n}_$i.log 2>&1 || exit 1
      GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality --lanes $n > $O/c5_q${q}_l${n}_$i.log 2>&1 || exit 1
    done
  done
done
for f in $O/c*_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
