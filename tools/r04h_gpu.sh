#!/bin/bash
# round 4: C5 wavefront A/B (majorant cell 8 / 16, tail threshold), C3 64-B node A/B, C5 wavefront profile
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04h
mkdir -p $O
for i in 1 2; do
  for v in c8 c16 c8t14 c8t18; do
    L=""; T=""
    [ $v = c16 ] && L=mitsuba-path-guiding_amd/build_cell16/libpgamd.so
    [ $v = c8t14 ] && T=16384
    [ $v = c8t18 ] && T=262144
    PG_LIB=$L PG_VOL_TAIL_PATHS=$T timeout -k 10 200 python bench.py --scene smoke --no-cpu > $O/c5_${v}_$i.log 2>&1 || { echo "c5 $v failed"; tail -5 $O/c5_${v}_$i.log; exit 1; }
    grep "^{" $O/c5_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c5 $v', d['value'], d['ms_per_step'], r['kernel'], r['frac'], {k: (v['avg_launch_ms'], v['frac'], v['time_share']) for k, v in r.get('kernels', {}).items()})"
  done
done
for i in 1 2 3; do
  for v in tri q64; do
    L=""; [ $v = q64 ] && L=mitsuba-path-guiding_amd/build_q64/libpgamd.so
    PG_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-quality > $O/c3_${v}_$i.log 2>&1 || { echo "bench $v failed"; tail -5 $O/c3_${v}_$i.log; exit 1; }
    grep "^{" $O/c3_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('c3 $v', d['value'], d['ms_per_step'], k['k_rays']['avg_launch_ms'], k['k_shade_all']['avg_launch_ms'])"
  done
done
timeout -k 10 400 bash tools/profile.sh gpurun_out/prof_r04h_c5 --scene smoke && python tools/pmc_summary.py gpurun_out/prof_r04h_c5 gpurun_out/r04h/c5 > $O/pmc_c5.txt 2>&1; cat $O/pmc_c5.txt | head -20
