#!/bin/bash
# round 4: C5 flight queues sorted by start cell (PG_VOL_SORT = min shard size; 0 = off), alternating;
# then the volume tests with sorting on
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04s
mkdir -p $O
PG_VOL_SORT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_volume.py -x -q --timeout 250 --timeout-method thread > $O/vol_tests_sorted.log 2>&1; s=$?; tail -2 $O/vol_tests_sorted.log; [ $s -eq 0 ] || exit 1
for r in 1 2; do
  for S in 0 1 4096; do
    PG_VOL_SORT=$S timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_s${S}_$r.log 2>&1 || { tail -5 $O/c5_s${S}_$r.log; exit 1; }
    grep "^{" $O/c5_s${S}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('sort $S run $r', d['value'], d['ms_per_step'], r['frac'], r.get('per_kernel', {}))" | cut -c1-600
  done
done
