#!/bin/bash
# round 4: C5 flight sort on / off with the split surface queues, alternating (3 runs each)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04af
mkdir -p $O
for r in 1 2 3; do
  for S in 4096 0; do
    PG_VOL_SORT=$S timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_s${S}_$r.log 2>&1 || { tail -5 $O/c5_s${S}_$r.log; exit 1; }
    grep "^{" $O/c5_s${S}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('sort $S run $r', d['value'], d['ms_per_step'], {n: v['avg_launch_ms'] for n, v in k.items()})"
  done
done
