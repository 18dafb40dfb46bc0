#!/bin/bash
# round 5 (ab): what contraction off costs now that it is off in every kernel: ab/fpcfast (make FPC=fast:
# kernels fast, volume kernels on) against the default build, C3 and C5 interleaved; the BSDF unit parity
# figures per material
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -rP -k bsdf_parity --timeout 250 --timeout-method thread > $O/bsdf.log 2>&1 || exit 1
grep -E "passed|failed|bsdf " $O/bsdf.log
for i in 1 2; do
  PG_LIB=ab/fpcfast/libpgamd.so timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_fast_$i.log 2>&1 || exit 1
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_off_$i.log 2>&1 || exit 1
  PG_LIB=ab/fpcfast/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_fast_$i.log 2>&1 || exit 1
  timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_off_$i.log 2>&1 || exit 1
done
for f in $O/c*_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('avg_launch_ms'), {n: (v.get('ms'), v.get('launches')) for n, v in r.get('kernels', {}).items()})"; done
