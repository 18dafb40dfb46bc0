#!/bin/bash
# round 5 (r): C3 register budgets with three lanes: k_shade_all at 5 waves (build_shade5), k_tail at 3
# (build_tail3), both (build_shade5tail3), against the default; alternating.  Then C5 at the new defaults.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05r
mkdir -p $O
L=mitsuba-path-guiding_amd
for i in 1 2; do
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_default_$i.log 2>&1 || exit 1
  for v in shade5 tail3 shade5tail3; do
    PG_LIB=$L/build_$v/libpgamd.so timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_${v}_$i.log 2>&1 || exit 1
  done
done
timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_default_1.log 2>&1 || exit 1
for f in $O/c3_*.log $O/c5_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], {n: v.get('ms') for n, v in r.get('kernels', {}).items()})"; done
