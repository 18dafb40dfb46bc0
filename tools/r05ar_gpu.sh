#!/bin/bash
# round 5 (ar): every hit in one shading class with run-time BSDF dispatch (ab/one, PG_ONE_CLASS=1; the queue
# then stays in rough slot order, so the SoA state reads coalesce) against the material-class queues: the C3
# variant's results differ from the class-queue build (parity_one.log, cause not investigated), then C3 x3
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05ar
mkdir -p $O
for i in 1 2 3; do
  PG_LIB=ab/one/libpgamd.so timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_one_$i.log 2>&1 || exit 1
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_cls_$i.log 2>&1 || exit 1
done
for f in $O/c*_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], {n: (v.get('ms'), v.get('traffic_over_algorithmic')) for n, v in r.get('kernels', {}).items()})"; done
