#!/bin/bash
# round 5 (a): GPU suite with the original-id tie rule + no FP contraction (tightened parity bars), then
# C3 / C5 A/B of FPC=off (build/) against FPC=fast (build_fast/), alternating runs on one box, then C5 with
# the transmittance walks inline (PG_VOL_NEE_STAGE=0) and with one interaction launch (PG_VOL_SPLIT_VERTEX=0)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rP --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?
grep -E "passed|failed|FAILED|c3 |c4 " $O/gpu_tests.log | head -20
[ $s -eq 0 ] || exit 1
L=mitsuba-path-guiding_amd
for i in 1 2; do
  PG_LIB=$L/build/libpgamd.so timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_off_$i.log 2>&1 || exit 1
  PG_LIB=$L/build_fast/libpgamd.so timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_fast_$i.log 2>&1 || exit 1
done
PG_LIB=$L/build/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_off_1.log 2>&1 || exit 1
PG_LIB=$L/build_fast/libpgamd.so timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_fast_1.log 2>&1 || exit 1
PG_VOL_NEE_STAGE=0 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_inline_1.log 2>&1 || exit 1
PG_VOL_SPLIT_VERTEX=0 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_nosplit_1.log 2>&1 || exit 1
for f in $O/c3_*.log $O/c5_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel'], r['frac'], {n: v.get('ms') for n, v in r.get('kernels', {}).items()})"; done
