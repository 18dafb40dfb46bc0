#!/bin/bash
# round 5 (y): fastlog without the library fallback (fewer spills): rounding probe; where free-flight
# distances still differ (tools/medium_mismatch.py); the C5 parity prints with the previous commit's
# library (device logf); C5 A/B head / new
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05y
mkdir -p $O
timeout -k 10 120 tools/log_rounding > $O/log_rounding.json 2>&1 || exit 1
cat $O/log_rounding.json
timeout -k 10 200 python tools/medium_mismatch.py $O/medium_mismatch.npz > $O/medium_mismatch.log 2>&1 || { tail -5 $O/medium_mismatch.log; exit 1; }
cat $O/medium_mismatch.log
PG_LIB=ab/head/libpgamd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_volume.py -m gpu -q -rP --timeout 250 --timeout-method thread > $O/vol_tests_head.log 2>&1
grep -E "passed|failed|FAILED|c5 |tracking" $O/vol_tests_head.log | head -20
for i in 1 2; do
  PG_LIB=ab/head/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_head_$i.log 2>&1 || exit 1
  timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_new_$i.log 2>&1 || exit 1
done
for f in $O/c*_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('avg_launch_ms'), {n: (v.get('ms'), v.get('launches')) for n, v in r.get('kernels', {}).items()})"; done
