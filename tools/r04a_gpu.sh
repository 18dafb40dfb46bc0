#!/bin/bash
# round 4 start: C3 and C5 bench lines at HEAD (baseline for this round's A/Bs)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 1; }
timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 1; }
for f in $O/bench_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"; done
