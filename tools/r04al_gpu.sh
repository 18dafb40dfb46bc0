#!/bin/bash
# round 4: C5 tail threshold 2^18 (default) / 2^17 / 2^19 with three lanes, alternating
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04al${SUFFIX:-}
mkdir -p $O
for r in 1 2; do
  for T in ${TAILS:-262144 131072 524288}; do
    PG_VOL_TAIL_PATHS=$T timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_t${T}_$r.log 2>&1 || { tail -5 $O/c5_t${T}_$r.log; exit 1; }
    grep "^{" $O/c5_t${T}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tail $T run $r', d['value'], d['ms_per_step'])"
  done
done
