#!/bin/bash
# round 5 (ac): surface launches specialised to diffuse / null materials (VolDev::models): GPU suite
# (tightened BSDF bars, the bit-identity test), then C5 with it (new) and without (PG_VOL_MODELS=0) and the
# previous commit's library (head), interleaved
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05ac
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rP --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?
grep -E "passed|failed|FAILED|c3 |c4 |c5 |tracking" $O/gpu_tests.log | head -30; [ $s -eq 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_new_$i.log 2>&1 || exit 1
  PG_VOL_MODELS=0 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_generic_$i.log 2>&1 || exit 1
  PG_LIB=ab/head/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_head_$i.log 2>&1 || exit 1
done
for f in $O/c*_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('avg_launch_ms'), {n: (v.get('ms'), v.get('launches')) for n, v in r.get('kernels', {}).items()})"; done
