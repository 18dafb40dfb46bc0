#!/bin/bash
# round 3: k_rays block order -- closest-hit blocks first (PG_RAYS_TRACE_FIRST=1) against shadow
# blocks first; C3 alternating runs + rank 0 of an 8-way shard
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03zg
mkdir -p $O
TF=mitsuba-path-guiding_amd/build_tf/libpgamd.so
bash tools/ab_bench.sh $O/c3 "" $TF || exit 1
for v in base tf; do
  L=""; [ $v = tf ] && L=$TF
  PG_LIB=$L timeout -k 10 300 python bench.py --scene kitchen --steps 2 --warmup 1 --no-cpu --no-quality > $O/kitchen_$v.log 2>&1 || exit 1
done
for f in $O/kitchen_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], {n: v['ms'] for n, v in d['roofline']['kernels'].items()})"; done
