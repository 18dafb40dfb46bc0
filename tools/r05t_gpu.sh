#!/bin/bash
# round 5 (t): C5 re-tune after the 3-wave kernels: tail threshold 2^16 / 2^17 (default) / 2^18, flight sort off
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05t
mkdir -p $O
for i in 1 2; do
  timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_default_$i.log 2>&1 || exit 1
  PG_VOL_TAIL_PATHS=65536 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_tail16_$i.log 2>&1 || exit 1
  PG_VOL_TAIL_PATHS=262144 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_tail18_$i.log 2>&1 || exit 1
  PG_VOL_SORT=0 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_nosort_$i.log 2>&1 || exit 1
done
for f in $O/c5_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], {n: v.get('ms') for n, v in r.get('kernels', {}).items()})"; done
