#!/bin/bash
# round 3 HEAD evidence after the 4-wide BVH: rocprofv3 kernel trace + FETCH/WRITE passes of the C3
# and C5 benches, the C3 counter passes (calibration stream), then the C3 and C5 bench lines
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/profile.sh gpurun_out/prof_r03zc && bash tools/profile.sh gpurun_out/prof_r03zc_c5 --scene smoke && echo profiles ok && \
bash tools/deep_profile.sh gpurun_out/deep_r03zc && python tools/deep_summary.py gpurun_out/deep_r03zc > gpurun_out/deep_r03zc/summary.json && echo deep ok || exit 1
O=gpurun_out/r03zc
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 1; }
timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 1; }
for f in $O/bench_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"; done
