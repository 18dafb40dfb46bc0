#!/bin/bash
# round 5 (ak): the jump grid also holds each leaf cell's meta record (sdMeta: the guided lookup's first load is its meta)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05ak
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rP --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?
grep -E "passed|failed|FAILED|c3 |c4 |c5 " $O/gpu_tests.log | head -20; [ $s -eq 0 ] || exit 1
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_new_$i.log 2>&1 || exit 1
  PG_LIB=ab/base/libpgamd.so timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_base_$i.log 2>&1 || exit 1
done
for i in 1 2; do
  timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_new_$i.log 2>&1 || exit 1
  PG_LIB=ab/base/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_base_$i.log 2>&1 || exit 1
done
for f in $O/c*_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('avg_launch_ms'), {n: (v.get('ms'), v.get('launches')) for n, v in r.get('kernels', {}).items()})"; done
