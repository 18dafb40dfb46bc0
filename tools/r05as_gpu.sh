#!/bin/bash
# round 5 (as): k_shade_all at 3 waves/SIMD (ab/w3, no scratch) against 4 (default, 12 B/lane of scratch), C3 x3
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05as
mkdir -p $O
for i in 1 2 3; do
  PG_LIB=ab/w3/libpgamd.so timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_w3_$i.log 2>&1 || exit 1
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_w4_$i.log 2>&1 || exit 1
done
for f in $O/c*_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], {n: v.get('ms') for n, v in r.get('kernels', {}).items()})"; done
