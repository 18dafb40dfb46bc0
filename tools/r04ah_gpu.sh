#!/bin/bash
# round 4: C5 with emitter surfaces in the cheap surface queue (build) against delta surfaces only
# (build_ab), alternating; the volume tests on the new build first
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04ah
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_volume.py -x -q --timeout 250 --timeout-method thread > $O/vol_tests.log 2>&1; s=$?; tail -2 $O/vol_tests.log; [ $s -eq 0 ] || exit 1
B=mitsuba-path-guiding_amd
for r in 1 2; do
  for b in build build_ab; do
    PG_LIB=$B/$b/libpgamd.so timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_${b}_$r.log 2>&1 || { tail -5 $O/c5_${b}_$r.log; exit 1; }
    grep "^{" $O/c5_${b}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('C5 $b run $r', d['value'], d['ms_per_step'], {n: v['avg_launch_ms'] for n, v in k.items()})"
  done
done
