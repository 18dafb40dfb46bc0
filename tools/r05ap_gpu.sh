#!/bin/bash
# round 5 (ap): C3 chunk-tail threshold re-measured on the current kernels (PG_TAIL_PATHS: 2^16 / 2^17 default /
# 2^18), x2 interleaved
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05ap
mkdir -p $O
for i in 1 2; do
  for t in 65536 default 262144; do
    if [ $t = default ]; then timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_${t}_$i.log 2>&1 || exit 1
    else PG_TAIL_PATHS=$t timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_${t}_$i.log 2>&1 || exit 1; fi
  done
done
for f in $O/c*_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])"; done
