#!/bin/bash
# round 3: strong-scaling rehearsal of rank 0's shard (W = 1..8), tail-threshold bench A/B, GPU suite
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03n
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal status $1 in $2"; exit 1;; esac; }
timeout -k 10 300 python -u tools/shard_timing.py 1,2,4,8 > $O/shard_timing.log 2>&1 || { s=$?; tail -5 $O/shard_timing.log; fatal $s shard; exit 1; }
cat $O/shard_timing.log
for i in 1 2; do
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/tail65k_$i.log 2>&1 || exit 1
  PG_TAIL_PATHS=131072 timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/tail131k_$i.log 2>&1 || exit 1
done
python - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r03n/tail*.log")):
    l = [x for x in open(f) if x.startswith("{")]
    if not l: print(f, "no result"); continue
    d = json.loads(l[-1])
    print(os.path.basename(f), d["value"], d["ms_per_step"])
PY
export TMPDIR=/tmp
for v in base corners; do
  L=""; [ $v = base ] && L=mitsuba-path-guiding_amd/build_base/libpgamd.so
  PG_LIB=$L timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -T -d $O/fetch_$v -o run --output-format csv -- python3 bench.py --scene smoke --steps 1 --warmup 0 --no-cpu --no-quality > $O/fetch_$v.log 2>&1 || { echo "fetch $v failed"; exit 1; }
done
python - <<'PY'
import csv, glob
for v in ("base", "corners"):
    tot, n = 0.0, 0
    for f in glob.glob(f"gpurun_out/r03n/fetch_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_volpath" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
                tot += float(r["Counter_Value"]); n += 1
    print(v, "k_volpath FETCH_SIZE KiB per launch", tot / max(n, 1), "launches", n)
PY
rocprofv3 --list-avail > $O/list_avail.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; tail -4 $O/gpu_tests.log
