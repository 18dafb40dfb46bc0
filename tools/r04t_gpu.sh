#!/bin/bash
# round 4: C5 with sorting on -- flight sort keys 16^3 cells (build) vs octant + 8^3 cells (build_ab),
# k_vflight at 4 waves/SIMD (build_ab2), tail threshold 2^17; alternating
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04t
mkdir -p $O
B=mitsuba-path-guiding_amd
for r in 1 2; do
  for cfg in "build 262144" "build_ab 262144" "build_ab2 262144" "build 131072"; do
    set -- $cfg
    PG_LIB=$B/$1/libpgamd.so PG_VOL_SORT=1 PG_VOL_TAIL_PATHS=$2 timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_$1_$2_$r.log 2>&1 || { tail -5 $O/c5_$1_$2_$r.log; exit 1; }
    grep "^{" $O/c5_$1_$2_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 tail $2 run $r', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
