#!/bin/bash
# round 3: block-private splat (PG_SPLAT_LDS) and tail-threshold A/B; splat/tree bit-identity tests
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03j
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal status $1 in $2"; exit 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_learned_fraction.py tests/test_gpu_comm.py tests/test_gpu_tail.py tests/test_gpu_volume.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; s=$?; tail -4 $O/tests.log; fatal $s tests
[ $s -eq 0 ] || exit 1
for w in 8 1; do for l in 0 1; do
  PG_SPLAT_LDS=$l PG_TRAIN_ONLY=1 PG_TRAIN_REPS=3 timeout -k 10 200 python -u tools/train_timing.py $w > $O/train_w${w}_lds$l.log 2>&1 || { fatal $? train; exit 1; }
  echo "W=$w lds=$l"; grep "rep 2" $O/train_w${w}_lds$l.log
done; done
for t in 16384 32768 131072; do
  PG_TAIL_PATHS=$t PG_TRAIN_ONLY=1 PG_TRAIN_REPS=3 timeout -k 10 200 python -u tools/train_timing.py 8 > $O/train_w8_tail$t.log 2>&1 || { fatal $? train; exit 1; }
  echo "W=8 tail=$t"; grep "rep 2" $O/train_w8_tail$t.log
done
for i in 1 2; do
  PG_SPLAT_LDS=0 timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/bench_lds0_$i.log 2>&1 || exit 1
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/bench_lds1_$i.log 2>&1 || exit 1
done
python - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r03j/bench_*.log")):
    l = [x for x in open(f) if x.startswith("{")]
    if not l: print(f, "no result"); continue
    d = json.loads(l[-1])
    print(os.path.basename(f), d["value"], d["ms_per_step"])
PY
