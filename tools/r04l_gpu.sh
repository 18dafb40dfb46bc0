#!/bin/bash
# round 4: k_rays occupancy A/B (8 waves with 40 B/lane of scratch, 7 and 6 without)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04l
mkdir -p $O
for i in 1 2 3; do
  for v in w8 w7 w6; do
    L=""
    [ $v = w7 ] && L=mitsuba-path-guiding_amd/build_rw7/libpgamd.so
    [ $v = w6 ] && L=mitsuba-path-guiding_amd/build_rw6/libpgamd.so
    PG_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-quality > $O/c3_${v}_$i.log 2>&1 || { echo "bench $v failed"; tail -5 $O/c3_${v}_$i.log; exit 1; }
    grep "^{" $O/c3_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('c3 $v', d['value'], d['ms_per_step'], k['k_rays']['avg_launch_ms'], k['k_shade_all']['avg_launch_ms'], k['k_trace']['avg_launch_ms'])"
  done
done
