#!/bin/bash
# round 3: shadow rays on the 4-wide BVH (PG_SHADOW4) against the 8-wide quantised BVH, with the
# 4-wide closest-hit BVH as the new default: GPU suite on both, det_check identity, C3 / kitchen / C5 A/B
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03zb
mkdir -p $O
B4=mitsuba-path-guiding_amd/build_bvh4s/libpgamd.so
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_base.log 2>&1 || { tail -3 $O/gpu_tests_base.log; exit 1; }
PG_LIB=$B4 timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_shadow4.log 2>&1; s=$?; tail -3 $O/gpu_tests_shadow4.log; [ $s -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/det_check.py --runs 1 > $O/det_base.log 2>&1 || exit 1
PG_LIB=$B4 timeout -k 10 200 python -u tools/det_check.py --runs 1 > $O/det_shadow4.log 2>&1 || exit 1
if diff <(grep "^run" $O/det_base.log) <(grep "^run" $O/det_shadow4.log) > /dev/null; then echo "det: identical"; else echo "det: DIFFERENT"; fi
bash tools/ab_bench.sh $O/c3 "" $B4 || exit 1
for v in base shadow4; do
  L=""; [ $v = shadow4 ] && L=$B4
  PG_LIB=$L timeout -k 10 300 python bench.py --scene kitchen --steps 2 --warmup 1 --no-cpu --no-quality > $O/kitchen_$v.log 2>&1 || exit 1
  PG_LIB=$L timeout -k 10 300 python bench.py --scene smoke --steps 2 --warmup 1 --no-cpu > $O/c5_$v.log 2>&1 || exit 1
done
for f in $O/kitchen_*.log $O/c5_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
