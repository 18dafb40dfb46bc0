#!/bin/bash
# round 4: blocked triangle records (PG_TRI_BLOCK, build_ab) -- the parity tests on that build, then C3
# and C5 against the default build, alternating
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04w
mkdir -p $O
B=mitsuba-path-guiding_amd
PG_LIB=$B/build_ab/libpgamd.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_volume.py -x -q --timeout 250 --timeout-method thread > $O/tests_block.log 2>&1; s=$?; tail -2 $O/tests_block.log; [ $s -eq 0 ] || exit 1
for r in 1 2; do
  for b in build build_ab; do
    PG_LIB=$B/$b/libpgamd.so timeout -k 10 300 python bench.py --no-cpu --no-quality > $O/c3_${b}_$r.log 2>&1 || { tail -5 $O/c3_${b}_$r.log; exit 1; }
    grep "^{" $O/c3_${b}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']['k_rays']; print('C3 $b run $r', d['value'], d['ms_per_step'], 'k_rays', k['avg_launch_ms'])"
  done
done
for b in build build_ab; do
  PG_LIB=$B/$b/libpgamd.so timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_${b}.log 2>&1 || { tail -5 $O/c5_${b}.log; exit 1; }
  grep "^{" $O/c5_${b}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 $b', d['value'], d['ms_per_step'])"
done
