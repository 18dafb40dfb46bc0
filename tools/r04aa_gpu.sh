#!/bin/bash
# round 4: k_rays leaf tests re-reading the ray (PG_TRACE_RELOAD, build_ab: 32 instead of 40 B/lane of
# scratch) against the default build on C3, alternating; the trace parity tests on build_ab first
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04aa
mkdir -p $O
B=mitsuba-path-guiding_amd
PG_LIB=$B/build_ab/libpgamd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread > $O/tests_reload.log 2>&1; s=$?; tail -2 $O/tests_reload.log; [ $s -eq 0 ] || exit 1
for r in 1 2 3; do
  for b in build build_ab; do
    PG_LIB=$B/$b/libpgamd.so timeout -k 10 300 python bench.py --no-cpu --no-quality > $O/c3_${b}_$r.log 2>&1 || { tail -5 $O/c3_${b}_$r.log; exit 1; }
    grep "^{" $O/c3_${b}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']['k_rays']; print('C3 $b run $r', d['value'], d['ms_per_step'], 'k_rays', k['avg_launch_ms'])"
  done
done
