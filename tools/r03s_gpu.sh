#!/bin/bash
# round 3: one-piece SD-tree upload/download + device jump grid: GPU suite, W=8 training timing, shard timing
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03s
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal status $1 in $2"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?; tail -4 $O/gpu_tests.log; fatal $s tests
[ $s -eq 0 ] || exit 1
PG_TRAIN_ONLY=1 PG_TRAIN_REPS=3 PG_DEBUG_REFIT=1 timeout -k 10 200 python -u tools/train_timing.py 8 > $O/train_w8.log 2>&1 || exit 1
grep "rep 2" $O/train_w8.log; grep "^refit" $O/train_w8.log | tail -5
timeout -k 10 300 python -u tools/shard_timing.py 1,8 > $O/shard_timing.log 2>&1 || exit 1
cat $O/shard_timing.log
for i in 1 2; do
  PG_LIB=mitsuba-path-guiding_amd/build_base/libpgamd.so timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/bench_base_$i.log 2>&1 || exit 1
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/bench_new_$i.log 2>&1 || exit 1
done
python - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r03s/bench_*.log")):
    l = [x for x in open(f) if x.startswith("{")]
    if not l: print(f, "no result"); continue
    d = json.loads(l[-1]); k = d["roofline"]["kernels"]
    print(os.path.basename(f), d["value"], d["ms_per_step"], {n: (v["ms"], v.get("frac")) for n, v in k.items()})
PY
