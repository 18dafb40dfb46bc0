#!/bin/bash
# round 5 (x): the kernels' own fastlog (csrc/pg_fastmath.h: the double log in ~20 FP64 operations):
# rounding probe over every tracking argument, GPU suite, then same-box A/B on C5 (head = device logf,
# dbl = the device library's double log, new) and C3 (head, new), interleaved
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 120 tools/log_rounding > $O/log_rounding.json 2>&1 || exit 1
cat $O/log_rounding.json
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rP --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?
grep -E "passed|failed|FAILED|c3 |c4 |c5 |tracking" $O/gpu_tests.log | head -30; [ $s -eq 0 ] || exit 1
for i in 1 2; do
  PG_LIB=ab/head/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_head_$i.log 2>&1 || exit 1
  timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_new_$i.log 2>&1 || exit 1
  PG_LIB=ab/dbl/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_dbl_$i.log 2>&1 || exit 1
  PG_LIB=ab/head/libpgamd.so timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_head_$i.log 2>&1 || exit 1
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_new_$i.log 2>&1 || exit 1
done
for f in $O/c*_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('avg_launch_ms'), {n: (v.get('ms'), v.get('launches')) for n, v in r.get('kernels', {}).items()})"; done
