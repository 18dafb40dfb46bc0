#!/bin/bash
# round 3: rocprofv3 kernel trace + FETCH/WRITE passes + deep counters of the C3 bench at HEAD
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/profile.sh gpurun_out/prof_r03b && bash tools/deep_profile.sh gpurun_out/deep_r03b && python tools/deep_summary.py gpurun_out/deep_r03b > gpurun_out/deep_r03b/summary.json && echo ok
