#!/bin/bash
# round 5 checkpoint 2 (C5 kernels changed): GPU suite, smoke(), the C5 profile (trace at the bench's steps +
# counter passes -> pmc_volpath_latest.json) and the C5 bench line with its CPU baseline, one call
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rP --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?
grep -E "passed|failed|FAILED|c3 |c4 " $O/gpu_tests.log | head; [ $s -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "c5 profile"
timeout -k 10 600 bash tools/profile.sh gpurun_out/prof_r05u_c5 --scene smoke && python tools/pmc_summary.py gpurun_out/prof_r05u_c5 $O/c5 > $O/c5_summary.txt 2>&1 || { echo "c5 profile failed"; exit 1; }
head -4 $O/c5_summary.txt
cp $O/pmc_volpath_latest.json profiles/pmc_volpath_latest.json
echo "c5 bench"
timeout -k 10 420 python bench.py --scene smoke > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 1; }
grep "^{" $O/bench_c5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; c=d.get('cpu_baseline') or {}; print('c5', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('frac_rocprof'), r.get('avg_launch_ms'), r.get('avg_launch_ms_rocprof'), r.get('traffic_over_algorithmic'), 'cpu', c.get('value'), c.get('cores'))"
