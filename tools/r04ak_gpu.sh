#!/bin/bash
# round 4 end: C5 rocprofv3 trace + HBM counter passes at HEAD (pmc_volpath_latest.json), then the GPU
# suite, smoke() and both bench lines.  usage: PG_REVISION=<hash> tools/r04ai_gpu.sh
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04ak
mkdir -p $O
timeout -k 10 420 bash tools/profile.sh gpurun_out/prof_r04ak_c5 --scene smoke && python tools/pmc_summary.py gpurun_out/prof_r04ak_c5 $O/c5 > $O/c5_summary.txt 2>&1 || { echo "c5 profile failed"; exit 1; }
cp $O/pmc_volpath_latest.json profiles/pmc_volpath_latest.json
head -4 $O/c5_summary.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?; grep -E "passed|failed|FAILED" $O/gpu_tests.log | head; [ $s -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 1; }
timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 1; }
for f in $O/bench_c3.log $O/bench_c5.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('frac_rocprof'), r.get('traffic_over_algorithmic'))"; done
