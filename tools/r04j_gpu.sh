#!/bin/bash
# round 4 checkpoint: full GPU suite, smoke, C3 and C5 bench lines at HEAD, the guiding breakdown
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?; grep -E "passed|failed|FAILED" $O/gpu_tests.log | head; [ $s -eq 0 ] || [ $s -eq 1 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 1; }
timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 1; }
for f in $O/bench_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"; done
timeout -k 10 400 python -u tools/guiding_breakdown_c3.py $O/guiding_breakdown.json > $O/guiding_breakdown.log 2>&1; s=$?; cut -c1-700 $O/guiding_breakdown.log; [ $s -eq 0 ] || exit 1
