#!/bin/bash
# round 5 (h): where the round-4 vs round-5 C5 difference comes from: one lane; no tail kernel
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05h
mkdir -p $O
R4=ab/r04/mitsuba-path-guiding_amd/build/libpgamd.so
PG_VOL_LANES=1 PG_LIB=$R4 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality --steps 2 > $O/c5_r04_lane1.log 2>&1 || exit 1
PG_VOL_LANES=1 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality --steps 2 > $O/c5_r05_lane1.log 2>&1 || exit 1
PG_VOL_TAIL_PATHS=0 PG_LIB=$R4 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality --steps 2 > $O/c5_r04_notail.log 2>&1 || exit 1
PG_VOL_TAIL_PATHS=0 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality --steps 2 > $O/c5_r05_notail.log 2>&1 || exit 1
PG_LIB=$R4 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality --steps 2 --train 0 > $O/c5_r04_notrain.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality --steps 2 --train 0 > $O/c5_r05_notrain.log 2>&1 || exit 1
for f in $O/c5_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], {n: v.get('ms') for n, v in r.get('kernels', {}).items()})"; done
