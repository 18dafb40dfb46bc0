#!/bin/bash
# round 5 (p): C5 interaction launches: medium at 3 waves (default) against the surface launch at 3 waves too
# (build_vs3) and the medium launch at 4 (build_vm4), alternating
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05p
mkdir -p $O
L=mitsuba-path-guiding_amd
for i in 1 2; do
  timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_default_$i.log 2>&1 || exit 1
  PG_LIB=$L/build_vs3/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_vs3_$i.log 2>&1 || exit 1
  PG_LIB=$L/build_vm4/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_vm4_$i.log 2>&1 || exit 1
done
for f in $O/c5_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], {n: v.get('ms') for n, v in r.get('kernels', {}).items()})"; done
