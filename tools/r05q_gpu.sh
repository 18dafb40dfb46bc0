#!/bin/bash
# round 5 (q): C5 register budgets of the interaction launches and the tail (builds build_<variant>), alternating
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05q
mkdir -p $O
L=mitsuba-path-guiding_amd
for i in 1 2; do
  for v in vs3 vs3vm4 vs4 vs3t3; do
    PG_LIB=$L/build_$v/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_${v}_$i.log 2>&1 || exit 1
  done
done
for f in $O/c5_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], {n: v.get('ms') for n, v in r.get('kernels', {}).items()})"; done
