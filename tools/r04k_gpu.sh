#!/bin/bash
# round 4: rocprofv3 kernel traces and HBM counter passes of the C3 and C5 bench commands at this revision
set -o pipefail
cd "$(dirname "$0")/.."
export PG_REVISION=0ae56edcfffe
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 500 bash tools/profile.sh gpurun_out/prof_r04k_c3 && python tools/pmc_summary.py gpurun_out/prof_r04k_c3 $O/c3 > $O/c3_summary.txt 2>&1; s=$?; head -12 $O/c3_summary.txt; [ $s -eq 0 ] || exit 1
timeout -k 10 400 bash tools/profile.sh gpurun_out/prof_r04k_c5 --scene smoke && python tools/pmc_summary.py gpurun_out/prof_r04k_c5 $O/c5 > $O/c5_summary.txt 2>&1; s=$?; head -12 $O/c5_summary.txt; [ $s -eq 0 ] || exit 1
