#!/bin/bash
# round 3: fp32 division and sqrt without correct rounding in the kernels (build_fd:
# -fno-hip-fp32-correctly-rounded-divide-sqrt with correctly rounded splat and triangle divisions; 60.3 k -> 48.6 k)
# against HEAD: GPU suite on the variant, C3 alternating runs, kitchen, C5
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03zo
mkdir -p $O
FD=mitsuba-path-guiding_amd/build_fd2/libpgamd.so
PG_LIB=$FD timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gpu_tests_fd.log 2>&1; s=$?; tail -3 $O/gpu_tests_fd.log; [ $s -eq 0 ] || exit 1
bash tools/ab_bench.sh $O/c3 "" $FD || exit 1
for v in base fd; do
  L=""; [ $v = fd ] && L=$FD
  PG_LIB=$L timeout -k 10 300 python bench.py --scene kitchen --steps 2 --warmup 1 --no-cpu --no-quality > $O/kitchen_$v.log 2>&1 || exit 1
  PG_LIB=$L timeout -k 10 300 python bench.py --scene smoke --steps 2 --warmup 1 --no-cpu > $O/c5_$v.log 2>&1 || exit 1
done
for f in $O/kitchen_*.log $O/c5_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
