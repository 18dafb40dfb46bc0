#!/bin/bash
# round 3: C3 bench line with the paired (same-tree) GPU/CPU RMSE ratio
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03zm
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 1; }
grep "^{" $O/bench_c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['rmse_vs_cpu']))"
