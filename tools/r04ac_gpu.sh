#!/bin/bash
# round 4: C5 recording passes on two lanes (default) vs one (PG_VOL_REC_LANES=1), alternating; volume tests first
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04ac
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_volume.py -x -q --timeout 250 --timeout-method thread > $O/vol_tests.log 2>&1; s=$?; tail -2 $O/vol_tests.log; [ $s -eq 0 ] || exit 1
for r in 1 2; do
  for L in 2 1; do
    PG_VOL_REC_LANES=$L timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_rec${L}_$r.log 2>&1 || { tail -5 $O/c5_rec${L}_$r.log; exit 1; }
    grep "^{" $O/c5_rec${L}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 rec lanes $L run $r', d['value'], d['ms_per_step'])"
  done
done
