#!/bin/bash
# round 4: volumetric wavefront lanes -- volume GPU tests, then C5 with 1 / 2 / 3 lanes (alternating)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_volume.py tests/test_gpu_configs.py -x -q --timeout 250 --timeout-method thread > $O/vol_tests.log 2>&1; s=$?; tail -3 $O/vol_tests.log; [ $s -eq 0 ] || exit 1
for r in 1 2; do
  for L in 1 3 2; do
    PG_VOL_LANES=$L timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_l${L}_$r.log 2>&1 || { tail -5 $O/c5_l${L}_$r.log; exit 1; }
    grep "^{" $O/c5_l${L}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lanes $L run $r', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
