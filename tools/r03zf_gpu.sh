#!/bin/bash
# round 3: the bench's own rank launcher (bench.py --gpus N without torchrun) on one MI355X, ranks
# sharing the GPU through the gloo rehearsal backend (RCCL refuses two ranks on one device)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03zf
mkdir -p $O
PG_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --quick > $O/gloo2_quick.log 2>&1 || { tail -5 $O/gloo2_quick.log; exit 1; }
PG_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --no-cpu --no-quality > $O/gloo2_c3.log 2>&1 || { tail -5 $O/gloo2_c3.log; exit 1; }
PG_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 4 --no-cpu --no-quality > $O/gloo4_c3.log 2>&1 || { tail -5 $O/gloo4_c3.log; exit 1; }
for f in $O/gloo*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['n_gpus'], d['value'], d['ms_per_step'], d['config']['parallelism'])"; done
