#!/bin/bash
# round 4: robust oracle walk -> same-tree divergence diagnosis on C3, k_tail grid cap check, C3 bench
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tail.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?; tail -3 $O/gpu_tests.log; [ $s -eq 0 ] || exit 1
timeout -k 10 700 python -u tools/diverge_c3.py $O/diverge.json > $O/diverge.log 2>&1 || { tail -5 $O/diverge.log; exit 1; }
head -c 3000 $O/diverge.log
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 1; }
grep "^{" $O/bench_c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], json.dumps(d['rmse_vs_cpu']['same_tree']))"
