#!/bin/bash
# round 4: volumetric wavefront -- bit-identity with the megakernel, volume GPU tests, C5 bench A/B
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_volume.py tests/test_gpu_bidir_pin.py -x -v --timeout 200 --timeout-method thread > $O/gpu_vol_tests.log 2>&1; s=$?; grep -E "PASS|FAIL|Error|passed|failed" $O/gpu_vol_tests.log | tail -25; [ $s -eq 0 ] || exit 1
for i in 1 2; do
  for wf in 1 0; do
    PG_VOL_WAVEFRONT=$wf timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_wf${wf}_$i.log 2>&1 || { echo "bench wf=$wf failed"; tail -5 $O/c5_wf${wf}_$i.log; exit 1; }
    grep "^{" $O/c5_wf${wf}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 wf=$wf', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
