#!/bin/bash
# round 4: C5 flight sort keys -- 16^3 cells vs octant + 8^3 cells (build_ab), sorting on; alternating
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04t
mkdir -p $O
for r in 1 2; do
  for K in cell oct; do
    L=mitsuba-path-guiding_amd/build/libpgamd.so; [ $K = oct ] && L=mitsuba-path-guiding_amd/build_ab/libpgamd.so
    PG_LIB=$L PG_VOL_SORT=1 timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_${K}_${r}.log 2>&1 || { tail -5 $O/c5_${K}_${r}.log; exit 1; }
    grep "^{" $O/c5_${K}_${r}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('key $K run $r', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
