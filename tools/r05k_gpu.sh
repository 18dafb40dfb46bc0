#!/bin/bash
# round 5 (k): the 4-wide BVH's breadth-first top levels (21 nodes) staged in LDS by k_rays' and k_trace's
# closest-hit blocks (build_ldstop: PG_RAYS_LDS_TOP=1 PG_TRACE_LDS_TOP=1) against the default, C3, alternating;
# the GPU trace parity tests on the variant
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05k
mkdir -p $O
L=mitsuba-path-guiding_amd
PG_LIB=$L/build_ldstop/libpgamd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -k "trace or bidir or cornell" --timeout 250 --timeout-method thread > $O/ldstop_tests.log 2>&1; s=$?; tail -2 $O/ldstop_tests.log; [ $s -eq 0 ] || exit 1
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_default_$i.log 2>&1 || exit 1
  PG_LIB=$L/build_ldstop/libpgamd.so timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_ldstop_$i.log 2>&1 || exit 1
done
for f in $O/c3_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], {n: v.get('ms') for n, v in r.get('kernels', {}).items()})"; done
