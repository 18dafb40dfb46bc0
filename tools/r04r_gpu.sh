#!/bin/bash
# round 4: C5 with 2 wavefront lanes -- tail threshold 2^18 / 2^19 / 2^20 and chunk 2^25 / 2^24 (alternating)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04r
mkdir -p $O
for r in 1 2; do
  for cfg in "18 0" "19 0" "20 0" "18 16777216" "19 16777216"; do
    set -- $cfg
    PG_VOL_TAIL_PATHS=$((1 << $1)) timeout -k 10 300 python bench.py --scene smoke --no-cpu --paths-in-flight $2 > $O/c5_t$1_c$2_$r.log 2>&1 || { tail -5 $O/c5_t$1_c$2_$r.log; exit 1; }
    grep "^{" $O/c5_t$1_c$2_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tail 2^$1 chunk $2 run $r', d['value'], d['ms_per_step'])"
  done
done
