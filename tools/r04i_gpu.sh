#!/bin/bash
# round 4: 64-B nodes default -> parity tests; C5 majorant cell 8 / 16 / 32 and tail threshold A/B on the
# wavefront; then the paired RMSE ratio and the guiding breakdown
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_volume.py -q --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?; grep -E "passed|failed|FAILED" $O/gpu_tests.log | head; [ $s -eq 0 ] || [ $s -eq 1 ] || exit 1
for i in 1 2; do
  for v in c8 c16 c32 c16t18; do
    L=""; T=""
    [ $v = c16 ] && L=mitsuba-path-guiding_amd/build_cell16/libpgamd.so
    [ $v = c32 ] && L=mitsuba-path-guiding_amd/build_cell32/libpgamd.so
    [ $v = c16t18 ] && L=mitsuba-path-guiding_amd/build_cell16/libpgamd.so && T=262144
    PG_LIB=$L PG_VOL_TAIL_PATHS=$T timeout -k 10 200 python bench.py --scene smoke --no-cpu > $O/c5_${v}_$i.log 2>&1 || { echo "c5 $v failed"; tail -5 $O/c5_${v}_$i.log; exit 1; }
    grep "^{" $O/c5_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c5 $v', d['value'], d['ms_per_step'], r['kernel'], r['frac'], d['pipeline']['algorithmic_bytes_per_step'])"
  done
done
timeout -k 10 420 python -u tools/rmse_paired_c3.py $O/rmse_paired.json --tiles 256 > $O/rmse_paired.log 2>&1; s=$?; tail -2 $O/rmse_paired.log; [ $s -eq 0 ] || exit 1
timeout -k 10 400 python -u tools/guiding_breakdown_c3.py $O/guiding_breakdown.json > $O/guiding_breakdown.log 2>&1; s=$?; cut -c1-600 $O/guiding_breakdown.log; [ $s -eq 0 ] || exit 1
