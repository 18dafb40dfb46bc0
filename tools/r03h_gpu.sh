#!/bin/bash
# round 3: counter passes over the C5 (smoke) bench
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/deep_profile.sh gpurun_out/deep_r03h_c5 --scene smoke && python tools/deep_summary.py gpurun_out/deep_r03h_c5 > gpurun_out/deep_r03h_c5/summary.json && echo deep ok
