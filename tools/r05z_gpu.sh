#!/bin/bash
# round 5 (z): contraction off in every kernel (pg_device.h no longer re-enables it after its region),
# microfacet / erf / erfinv on the reference's fastlog / fastexp, the tracking log switchable
# (PG_TRACK_FASTLOG, ab/exact): GPU suite, the volume tests with the exact tracking log, free-flight
# mismatches; same-box A/B against the previous commit's library on C3 and C5
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05z
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rP --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?
grep -E "passed|failed|FAILED|c3 |c4 |c5 |tracking" $O/gpu_tests.log | head -30; [ $s -eq 0 ] || exit 1
PG_LIB=ab/exact/libpgamd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_volume.py -m gpu -q -rP --timeout 250 --timeout-method thread > $O/vol_tests_exact.log 2>&1
grep -E "passed|failed|FAILED|c5 |tracking" $O/vol_tests_exact.log | head -20
PG_LIB=ab/exact/libpgamd.so timeout -k 10 200 python tools/medium_mismatch.py $O/medium_mismatch_exact.npz > $O/medium_mismatch_exact.log 2>&1 || exit 1
cat $O/medium_mismatch_exact.log
for i in 1 2; do
  PG_LIB=ab/head/libpgamd.so timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_head_$i.log 2>&1 || exit 1
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_new_$i.log 2>&1 || exit 1
  PG_LIB=ab/head/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_head_$i.log 2>&1 || exit 1
  timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_new_$i.log 2>&1 || exit 1
done
for f in $O/c*_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('avg_launch_ms'), {n: (v.get('ms'), v.get('launches')) for n, v in r.get('kernels', {}).items()})"; done
