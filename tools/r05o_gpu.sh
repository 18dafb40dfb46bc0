#!/bin/bash
# round 5 (o): C5 with the path state stored before the inline walks: one interaction launch (default) against
# medium / surface launches, the medium one at 2 (build) or 3 (build_vm3, 44 B/lane of scratch) waves/SIMD;
# then the GPU volume tests on the default build
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05o
mkdir -p $O
L=mitsuba-path-guiding_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_volume.py tests/test_gpu_bidir_pin.py -q --timeout 250 --timeout-method thread > $O/vol_tests.log 2>&1; s=$?; tail -2 $O/vol_tests.log; [ $s -eq 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_one_$i.log 2>&1 || exit 1
  PG_VOL_SPLIT_VERTEX=1 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_split2_$i.log 2>&1 || exit 1
  PG_VOL_SPLIT_VERTEX=1 PG_LIB=$L/build_vm3/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_split3_$i.log 2>&1 || exit 1
done
for f in $O/c5_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], {n: v.get('ms') for n, v in r.get('kernels', {}).items()})"; done
