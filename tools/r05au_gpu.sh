#!/bin/bash
# round 5 (au): per-class shading launches (PG_NO_SHADE_FUSION=1: each class kernel at its own register count,
# 96-127 VGPRs without scratch) against the fused k_shade_all (129 VGPRs, 12 B/lane of scratch at 4 waves), C3 x3
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05au
mkdir -p $O
for i in 1 2 3; do
  PG_NO_SHADE_FUSION=1 timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_class_$i.log 2>&1 || exit 1
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_fused_$i.log 2>&1 || exit 1
done
for f in $O/c*_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
