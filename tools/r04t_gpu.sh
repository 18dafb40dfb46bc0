#!/bin/bash
# round 4: C5 flight sort keys -- 16^3 cells vs octant + 8^3 cells (build_ab), and the tail threshold
# 2^16 / 2^17 with sorting on and two lanes; alternating
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04t
mkdir -p $O
for r in 1 2; do
  for cfg in "cell 262144" "oct 262144" "cell 131072" "cell 65536"; do
    set -- $cfg
    K=$1; T=$2
    L=mitsuba-path-guiding_amd/build/libpgamd.so; [ $K = oct ] && L=mitsuba-path-guiding_amd/build_ab/libpgamd.so
    PG_LIB=$L PG_VOL_SORT=1 PG_VOL_TAIL_PATHS=$T timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_${K}_${T}_${r}.log 2>&1 || { tail -5 $O/c5_${K}_${T}_${r}.log; exit 1; }
    grep "^{" $O/c5_${K}_${T}_${r}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('key $K tail $T run $r', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
