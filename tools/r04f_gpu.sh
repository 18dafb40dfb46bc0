#!/bin/bash
# round 4: TriAccel on the device (parity + A/B against Woop), volumetric wavefront (bit-identity + A/B),
# C5 index-check build, same-tree divergence with TriAccel
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_volume.py tests/test_gpu_tail.py tests/test_gpu_configs.py -q --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?; grep -E "passed|failed|FAILED" $O/gpu_tests.log | head -20; [ $s -eq 0 ] || [ $s -eq 1 ] || exit 1
for i in 1 2; do
  for v in tri woop q64; do
    L=""; [ $v = woop ] && L=mitsuba-path-guiding_amd/build_woop/libpgamd.so
    [ $v = q64 ] && L=mitsuba-path-guiding_amd/build_q64/libpgamd.so
    PG_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-quality > $O/c3_${v}_$i.log 2>&1 || { echo "bench $v failed"; tail -5 $O/c3_${v}_$i.log; exit 1; }
    grep "^{" $O/c3_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 $v', d['value'], d['ms_per_step'], d['roofline']['kernels']['k_rays']['avg_launch_ms'], d['segments_per_path'])"
  done
done
for i in 1 2; do
  for wf in 1 0; do
    PG_VOL_WAVEFRONT=$wf timeout -k 10 200 python bench.py --scene smoke --no-cpu > $O/c5_wf${wf}_$i.log 2>&1 || { echo "bench c5 wf=$wf failed"; tail -5 $O/c5_wf${wf}_$i.log; exit 1; }
    grep "^{" $O/c5_wf${wf}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 wf=$wf', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 300 python -u tools/volcheck_c5.py 1 > $O/volcheck.log 2>&1; s=$?; tail -2 $O/volcheck.log; [ $s -eq 0 ] || exit 1
timeout -k 10 400 python -u tools/diverge_c3.py $O/diverge.json --top 6 > $O/diverge.log 2>&1 || { tail -5 $O/diverge.log; exit 1; }
head -c 1500 $O/diverge.log
