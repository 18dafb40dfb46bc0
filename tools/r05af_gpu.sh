#!/bin/bash
# round 5 (af): triangle records' three rows loaded up front (PG_TRI_PRELOAD=1) against row by row
# (ab/nopre): trace parity, then C3 x3 and C5 x2 interleaved
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05af
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 250 --timeout-method thread > $O/parity.log 2>&1 || { tail -20 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_pre_$i.log 2>&1 || exit 1
  PG_LIB=ab/nopre/libpgamd.so timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_nopre_$i.log 2>&1 || exit 1
done
for i in 1 2; do
  timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_pre_$i.log 2>&1 || exit 1
  PG_LIB=ab/nopre/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_nopre_$i.log 2>&1 || exit 1
done
for f in $O/c*_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('avg_launch_ms'), {n: (v.get('ms'), v.get('launches')) for n, v in r.get('kernels', {}).items()})"; done
