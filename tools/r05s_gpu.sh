#!/bin/bash
# round 5 (s): C5 after the 3-wave interactions: the default (walks inline) against the k_vnee stage (its
# interaction launches at 3 waves too), k_vflight at 5 waves (build_vf5, 124 B/lane of scratch), 2 and 4 lanes
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05s
mkdir -p $O
L=mitsuba-path-guiding_amd
for i in 1 2; do
  timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_default_$i.log 2>&1 || exit 1
  PG_VOL_NEE_STAGE=1 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_stage_$i.log 2>&1 || exit 1
  PG_LIB=$L/build_vf5/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_vf5_$i.log 2>&1 || exit 1
done
PG_VOL_LANES=2 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_lanes2.log 2>&1 || exit 1
PG_VOL_LANES=4 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_lanes4.log 2>&1 || exit 1
for f in $O/c5_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], {n: v.get('ms') for n, v in r.get('kernels', {}).items()})"; done
