#!/bin/bash
# round 3: full bench lines at HEAD (C3 with quality + CPU baseline, C5, C2 Cornell, C4 kitchen on one GPU), smoke()
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 1; }
timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 1; }
timeout -k 10 200 python bench.py --scene cornell --width 512 --height 512 --no-cpu --no-quality > $O/bench_c2_cornell.log 2>&1 || { tail -5 $O/bench_c2_cornell.log; exit 1; }
timeout -k 10 300 python bench.py --scene kitchen --width 1920 --height 1080 --no-cpu --no-quality > $O/bench_c4_kitchen_1gpu.log 2>&1 || { tail -5 $O/bench_c4_kitchen_1gpu.log; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
for f in $O/bench_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'), (d.get('quality') or {}).get('guided_over_unguided'))"; done
tail -3 $O/smoke.log
