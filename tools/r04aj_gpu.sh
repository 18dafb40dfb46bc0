#!/bin/bash
# round 4: C5 with 3 / 4 wavefront lanes at the final kernels, alternating
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04aj${SUFFIX:-}
mkdir -p $O
for r in 1 2; do
  for L in 3 4; do
    PG_VOL_LANES=$L timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_l${L}_$r.log 2>&1 || { tail -5 $O/c5_l${L}_$r.log; exit 1; }
    grep "^{" $O/c5_l${L}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lanes $L run $r', d['value'], d['ms_per_step'])"
  done
done
