#!/bin/bash
# round 3 final HEAD evidence: rocprofv3 kernel trace + FETCH/WRITE passes of the C3 and C5 benches,
# summarised on the box (PG_REVISION = the uploaded HEAD) into profiles/ (pmc_latest.json, which the
# bench line reads) and copied to gpurun_out/r03zj_profiles; then the C3 counter passes
# usage: tools/r03zj_prof.sh REVISION
set -o pipefail
cd "$(dirname "$0")/.."
export PG_REVISION=$1
bash tools/profile.sh gpurun_out/prof_r03zj && bash tools/profile.sh gpurun_out/prof_r03zj_c5 --scene smoke && echo profiles ok || exit 1
python tools/pmc_summary.py gpurun_out/prof_r03zj profiles/r03zj && python tools/pmc_summary.py gpurun_out/prof_r03zj_c5 profiles/r03zj_c5 || exit 1
mkdir -p gpurun_out/r03zj_profiles && cp profiles/r03zj_* profiles/pmc_latest.json profiles/pmc_volpath_latest.json gpurun_out/r03zj_profiles/
bash tools/deep_profile.sh gpurun_out/deep_r03zj && python tools/deep_summary.py gpurun_out/deep_r03zj > gpurun_out/deep_r03zj/summary.json && echo deep ok
