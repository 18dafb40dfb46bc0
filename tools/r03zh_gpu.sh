#!/bin/bash
# round 3: camera rays without the implied throughput / prev stores and first-bounce shading without
# their loads (build_el) against HEAD: GPU suite on the variant, det_check identity, C3 alternating runs
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03zh
mkdir -p $O
EL=mitsuba-path-guiding_amd/build_el/libpgamd.so
PG_LIB=$EL timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/gpu_tests_el.log 2>&1; s=$?; tail -3 $O/gpu_tests_el.log; [ $s -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/det_check.py --runs 1 > $O/det_base.log 2>&1 || exit 1
PG_LIB=$EL timeout -k 10 200 python -u tools/det_check.py --runs 1 > $O/det_el.log 2>&1 || exit 1
if diff <(grep "^run" $O/det_base.log) <(grep "^run" $O/det_el.log) > /dev/null; then echo "det: identical"; else echo "det: DIFFERENT"; fi
bash tools/ab_bench.sh $O/c3 "" $EL || exit 1
