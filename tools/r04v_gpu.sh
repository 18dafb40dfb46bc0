#!/bin/bash
# round 4: C5 flight sort on / off at 4 k_vflight waves (alternating), then the HBM counters of C5 with sorting off
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04v
mkdir -p $O
for r in 1 2; do
  for S in 0 4096; do
    PG_VOL_SORT=$S timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_s${S}_$r.log 2>&1 || { tail -5 $O/c5_s${S}_$r.log; exit 1; }
    grep "^{" $O/c5_s${S}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sort $S run $r', d['value'], d['ms_per_step'])"
  done
done
PG_VOL_SORT=0 timeout -k 10 420 bash tools/profile.sh gpurun_out/prof_r04v_c5_nosort --scene smoke && python tools/pmc_summary.py gpurun_out/prof_r04v_c5_nosort $O/c5_nosort > $O/c5_nosort_summary.txt 2>&1 || exit 1
head -4 $O/c5_nosort_summary.txt
