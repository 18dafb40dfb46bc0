#!/bin/bash
# round 3 HEAD evidence: rocprofv3 kernel trace + FETCH/WRITE passes of the C3 and C5 benches, then
# the C3 counter passes (calibration stream)
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/profile.sh gpurun_out/prof_r03r && bash tools/profile.sh gpurun_out/prof_r03r_c5 --scene smoke && echo profiles ok && \
bash tools/deep_profile.sh gpurun_out/deep_r03r && python tools/deep_summary.py gpurun_out/deep_r03r > gpurun_out/deep_r03r/summary.json && echo deep ok
