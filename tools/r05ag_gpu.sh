#!/bin/bash
# round 5 (ag): closest hits on the 8-wide quantised BVH (ab/wide, PG_CLOSEST_WIDE=1, experiment) against the
# 4-wide walk: trace agreement on C3's own rays through the bench, C3 x3 interleaved
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05ag
mkdir -p $O
for i in 1 2 3; do
  PG_LIB=ab/wide/libpgamd.so timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_wide_$i.log 2>&1 || { tail -5 $O/c3_wide_$i.log; exit 1; }
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_bvh4_$i.log 2>&1 || exit 1
done
for f in $O/c*_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('avg_launch_ms'), {n: (v.get('ms'), v.get('launches')) for n, v in r.get('kernels', {}).items()})"; done
