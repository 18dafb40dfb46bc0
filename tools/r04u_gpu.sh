#!/bin/bash
# round 4: C3 lanes (2 / 3 / 4) and k_tail threshold (2^16 / 2^17 / 2^18) re-measured at this revision; alternating
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04u
mkdir -p $O
for r in 1 2; do
  for cfg in "3 131072" "2 131072" "4 131072" "3 65536" "3 262144"; do
    set -- $cfg
    PG_TAIL_PATHS=$2 timeout -k 10 300 python bench.py --no-cpu --no-quality --lanes $1 > $O/c3_l$1_t$2_$r.log 2>&1 || { tail -5 $O/c3_l$1_t$2_$r.log; exit 1; }
    grep "^{" $O/c3_l$1_t$2_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lanes $1 tail $2 run $r', d['value'], d['ms_per_step'])"
  done
done
