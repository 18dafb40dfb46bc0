#!/bin/bash
# round 5 (g): C5, the round-4 library against this tree's (inline walks, 7 state arrays per slot), alternating
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05g
mkdir -p $O
for i in 1 2; do
  PG_LIB=ab/r04/mitsuba-path-guiding_amd/build/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_r04_$i.log 2>&1 || exit 1
  timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_r05_$i.log 2>&1 || exit 1
done
for f in $O/c5_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], {n: v.get('ms') for n, v in r.get('kernels', {}).items()})"; done
