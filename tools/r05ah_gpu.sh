#!/bin/bash
# round 5 (ah): one-medium scenes read the medium record with scalar loads (PG_MED_UNIFORM=1) against per-lane
# loads (ab/nomu): volume tests, then C5 x3 interleaved
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05ah
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_volume.py -m gpu -q -rP --timeout 250 --timeout-method thread > $O/vol_tests.log 2>&1 || { tail -20 $O/vol_tests.log; exit 1; }
grep -E "passed|failed|c5 |tracking" $O/vol_tests.log
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_mu_$i.log 2>&1 || exit 1
  PG_LIB=ab/nomu/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_nomu_$i.log 2>&1 || exit 1
done
for f in $O/c*_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('avg_launch_ms'), {n: (v.get('ms'), v.get('launches')) for n, v in r.get('kernels', {}).items()})"; done
