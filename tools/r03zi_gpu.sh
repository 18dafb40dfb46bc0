#!/bin/bash
# round 3: robust slab test (per-axis padding, default) at 8 waves/SIMD for k_rays (28 B/lane of
# scratch) and at 7 (build_w7, no scratch) against no padding (build_nr): GPU suite on the default,
# det_check against build_nr, C3 alternating runs, kitchen
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03zi
mkdir -p $O
W7=mitsuba-path-guiding_amd/build_w7/libpgamd.so
NR=mitsuba-path-guiding_amd/build_nr/libpgamd.so
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?; tail -3 $O/gpu_tests.log; [ $s -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/det_check.py --runs 1 > $O/det_robust.log 2>&1 || exit 1
PG_LIB=$NR timeout -k 10 200 python -u tools/det_check.py --runs 1 > $O/det_nr.log 2>&1 || exit 1
if diff <(grep "^run" $O/det_robust.log) <(grep "^run" $O/det_nr.log) > /dev/null; then echo "det: identical"; else echo "det: DIFFERENT"; fi
for i in 1 2; do
  for v in robust w7 nr; do
    L=""; [ $v = w7 ] && L=$W7; [ $v = nr ] && L=$NR
    PG_LIB=$L timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_${v}_$i.log 2>&1 || exit 1
  done
done
for v in robust w7 nr; do
  L=""; [ $v = w7 ] && L=$W7; [ $v = nr ] && L=$NR
  PG_LIB=$L timeout -k 10 300 python bench.py --scene kitchen --steps 2 --warmup 1 --no-cpu --no-quality > $O/kitchen_$v.log 2>&1 || exit 1
done
PG_LIB=$W7 timeout -k 10 300 python bench.py --scene smoke --steps 2 --warmup 1 --no-cpu > $O/c5_w7.log 2>&1 || exit 1
for f in $O/c3_*.log $O/kitchen_*.log $O/c5_*.log; do grep "^{" $f | python -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline'].get('kernels',{})
print('$f', d['value'], d['ms_per_step'], {n: v['ms'] for n, v in k.items()})"; done
