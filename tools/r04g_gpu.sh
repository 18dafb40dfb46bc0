#!/bin/bash
# round 4: paired RMSE ratio by sample size (C3); guided vs unguided at equal time by pixel class
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 420 python -u tools/rmse_paired_c3.py $O/rmse_paired.json --tiles 256 > $O/rmse_paired.log 2>&1; s=$?; tail -3 $O/rmse_paired.log; [ $s -eq 0 ] || exit 1
timeout -k 10 500 python -u tools/guiding_breakdown_c3.py $O/guiding_breakdown.json > $O/guiding_breakdown.log 2>&1; s=$?; cut -c1-700 $O/guiding_breakdown.log; [ $s -eq 0 ] || exit 1
