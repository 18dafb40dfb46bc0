#!/bin/bash
# round 5 (at): final check of the tree as left for the round end: GPU suite, smoke(), the default bench line
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05at
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?
tail -1 $O/gpu_tests.log; [ $s -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 420 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep "^{" $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; c=d.get('cpu_baseline') or {}; print(d['metric'], d['value'], d['unit'], d['ms_per_step'], r['kernel'], r['frac'], r.get('frac_rocprof'), 'cpu', c.get('value'), c.get('cores'))"
