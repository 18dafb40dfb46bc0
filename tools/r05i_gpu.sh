#!/bin/bash
# round 5 (i): C5 walks inline against the k_vnee stage (no extra streams now), alternating; the overlap
# variant (a second stream per lane) once
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05i
mkdir -p $O
for i in 1 2; do
  timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_inline_$i.log 2>&1 || exit 1
  PG_VOL_NEE_STAGE=1 PG_VOL_NEE_OVERLAP=0 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_stage_$i.log 2>&1 || exit 1
done
PG_VOL_NEE_STAGE=1 PG_VOL_NEE_OVERLAP=1 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_overlap_1.log 2>&1 || exit 1
PG_VOL_NEE_STAGE=1 PG_VOL_NEE_OVERLAP=1 PG_VOL_LANES=2 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_overlap_lanes2.log 2>&1 || exit 1
for f in $O/c5_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], {n: v.get('ms') for n, v in r.get('kernels', {}).items()})"; done
