#!/bin/bash
# round 5 (j): hardware queues (GPU_MAX_HW_QUEUES, HIP's default 4 per process) against path lanes: C3 and C5
# with 3 and 4 lanes at 4 and 8 queues
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05j
mkdir -p $O
for q in 4 8; do
  for lanes in 3 4; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python bench.py --no-cpu --no-quality --lanes $lanes > $O/c3_q${q}_l${lanes}.log 2>&1 || exit 1
  done
done
for q in 4 8; do
  for lanes in 3 4; do
    GPU_MAX_HW_QUEUES=$q PG_VOL_LANES=$lanes timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_q${q}_l${lanes}.log 2>&1 || exit 1
  done
done
for f in $O/c3_*.log $O/c5_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
