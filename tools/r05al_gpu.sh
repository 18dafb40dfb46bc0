#!/bin/bash
# round 5 checkpoint 4 (the jump grid holding leaf D-tree ids): GPU suite, smoke(), per scene the profile + counter passes and the bench line with its CPU baseline
# (tools/profile.sh -> pmc_latest.json / pmc_volpath_latest.json) and the bench line with its CPU baseline,
# in one call so the line's HIP-event durations and the profile's come from the same box.
# usage: PG_REVISION=<hash> tools/r05al_gpu.sh
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05al
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rP --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?
grep -E "passed|failed|FAILED|c3 |c4 |c5 |bsdf " $O/gpu_tests.log | head -30; [ $s -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "c3 profile"
timeout -k 10 500 bash tools/profile.sh gpurun_out/prof_r05al_c3 && python tools/pmc_summary.py gpurun_out/prof_r05al_c3 $O/c3 > $O/c3_summary.txt 2>&1 || { echo "c3 profile failed"; exit 1; }
head -4 $O/c3_summary.txt
cp $O/pmc_latest.json profiles/pmc_latest.json
echo "c3 bench"
timeout -k 10 420 python bench.py > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 1; }
echo "c5 profile"
timeout -k 10 500 bash tools/profile.sh gpurun_out/prof_r05al_c5 --scene smoke && python tools/pmc_summary.py gpurun_out/prof_r05al_c5 $O/c5 > $O/c5_summary.txt 2>&1 || { echo "c5 profile failed"; exit 1; }
head -4 $O/c5_summary.txt
cp $O/pmc_volpath_latest.json profiles/pmc_volpath_latest.json
echo "c5 bench"
timeout -k 10 420 python bench.py --scene smoke > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 1; }
for f in $O/bench_c3.log $O/bench_c5.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; c=d.get('cpu_baseline') or {}; print('$f', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('frac_rocprof'), r.get('avg_launch_ms'), r.get('avg_launch_ms_rocprof'), r.get('traffic_over_algorithmic'), 'cpu', c.get('value'), c.get('cores'))"; done
