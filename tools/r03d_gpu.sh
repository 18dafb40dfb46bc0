#!/bin/bash
# round 3: learned-fraction debug, tail GPU tests, training timing with/without k_tail, C3 quality per
# fraction mode, GPU suite, ray-sort and tail bench A/B.  Any timeout / abort / segfault ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03d
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal status $1 in $2"; exit 1;; esac; }
timeout -k 10 120 python -u tools/dbg_learned.py > $O/dbg_learned.log 2>&1; s=$?; tail -20 $O/dbg_learned.log; fatal $s dbg
timeout -k 10 200 python -u -m pytest tests/test_gpu_tail.py -x -v --timeout 150 --timeout-method thread > $O/tail_test.log 2>&1; s=$?; tail -5 $O/tail_test.log; fatal $s tail_test
[ $s -eq 0 ] || exit 1
for t in -1 0; do
  PG_TAIL_PATHS=$([ $t = -1 ] && echo 0 || echo 65536) timeout -k 10 200 python -u tools/train_timing.py 8 > $O/train_w8_tail$t.log 2>&1 || { fatal $? train; exit 1; }
  echo "tail $t"; cat $O/train_w8_tail$t.log
done
for i in 1 2; do
  PG_TAIL_PATHS=0 timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/tail0_$i.log 2>&1 || exit 1
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/sort0_$i.log 2>&1 || exit 1
  PG_RAY_SORT=1 timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/sort1_$i.log 2>&1 || exit 1
done
python - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r03d/sort*.log") + glob.glob("gpurun_out/r03d/tail0_*.log")):
    l = [x for x in open(f) if x.startswith("{")]
    if not l: print(f, "no result"); continue
    d = json.loads(l[-1]); k = d["roofline"].get("kernels", {})
    print(os.path.basename(f), d["value"], d["ms_per_step"], {n: v["ms"] for n, v in k.items()})
PY
