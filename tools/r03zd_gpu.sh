#!/bin/bash
# round 3: SAH-optimal 4-wide collapse (default) against the greedy largest-area collapse
# (PG_BVH4_GREEDY=1): GPU suite, det_check identity, alternating C3 runs, kitchen and C5
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03zd
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?; tail -3 $O/gpu_tests.log; [ $s -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/det_check.py --runs 1 > $O/det_dp.log 2>&1 || exit 1
PG_BVH4_GREEDY=1 timeout -k 10 200 python -u tools/det_check.py --runs 1 > $O/det_greedy.log 2>&1 || exit 1
if diff <(grep "^run" $O/det_dp.log) <(grep "^run" $O/det_greedy.log) > /dev/null; then echo "det: identical"; else echo "det: DIFFERENT"; fi
for i in 1 2; do
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_dp_$i.log 2>&1 || exit 1
  PG_BVH4_GREEDY=1 timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_greedy_$i.log 2>&1 || exit 1
done
for v in dp greedy; do
  G=0; [ $v = greedy ] && G=1
  PG_BVH4_GREEDY=$G timeout -k 10 300 python bench.py --scene kitchen --steps 2 --warmup 1 --no-cpu --no-quality > $O/kitchen_$v.log 2>&1 || exit 1
  PG_BVH4_GREEDY=$G timeout -k 10 300 python bench.py --scene smoke --steps 2 --warmup 1 --no-cpu > $O/c5_$v.log 2>&1 || exit 1
done
for f in $O/c3_*.log $O/kitchen_*.log $O/c5_*.log; do grep "^{" $f | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline'].get('kernels',{})
print('$f', d['value'], d['ms_per_step'], {n: v['ms'] for n, v in k.items()})"; done
