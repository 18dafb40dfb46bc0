#!/bin/bash
# round 5 (d): non-temporal path-state loads/stores (PG_NT_STATE=1, build_nt/) -- run-to-run determinism of
# the guided kitchen training with three lanes (tools/det_kitchen.py) and C3 A/B against the default build;
# C5 with one interaction launch (PG_VOL_SPLIT_VERTEX=0) against two, walks inline
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05d
mkdir -p $O
L=mitsuba-path-guiding_amd
PG_LIB=$L/build_nt/libpgamd.so timeout -k 10 300 python tools/det_kitchen.py --lanes 3 --reps 6 > $O/det_nt.log 2>&1 || exit 1
tail -3 $O/det_nt.log
PG_LIB=$L/build/libpgamd.so timeout -k 10 300 python tools/det_kitchen.py --lanes 3 --reps 4 > $O/det_default.log 2>&1 || exit 1
tail -3 $O/det_default.log
for i in 1 2; do
  PG_LIB=$L/build/libpgamd.so timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_default_$i.log 2>&1 || exit 1
  PG_LIB=$L/build_nt/libpgamd.so timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_nt_$i.log 2>&1 || exit 1
done
for i in 1 2; do
  timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_split_$i.log 2>&1 || exit 1
  PG_VOL_SPLIT_VERTEX=0 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_nosplit_$i.log 2>&1 || exit 1
done
for f in $O/c3_*.log $O/c5_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], {n: v.get('ms') for n, v in r.get('kernels', {}).items()})"; done
