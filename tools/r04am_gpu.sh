#!/bin/bash
# round 4 end: GPU suite, smoke() and both bench lines at HEAD (kernels as profiled in r04ak)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04am
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?; grep -E "passed|failed|FAILED" $O/gpu_tests.log | head; [ $s -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 1; }
timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 1; }
for f in $O/bench_c3.log $O/bench_c5.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('frac_rocprof'))"; done
