#!/bin/bash
# C5 A/B of two builds (alternating) + FETCH_SIZE pass of build B: tools/ab_c5.sh OUT LIB_A LIB_B
set -eo pipefail
OUT=$1; A=$2; B=$3
mkdir -p "$OUT"
for i in 1 2; do
  PG_LIB=$A timeout -k 10 200 python bench.py --scene smoke --steps 2 --warmup 1 --no-cpu > "$OUT/a_$i.log" 2>&1
  PG_LIB=$B timeout -k 10 200 python bench.py --scene smoke --steps 2 --warmup 1 --no-cpu > "$OUT/b_$i.log" 2>&1
done
export TMPDIR=/tmp
PG_LIB=$B timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch_b" -o run --output-format csv -- python3 bench.py --scene smoke --steps 1 --warmup 0 --no-cpu > "$OUT/fetch_b.log" 2>&1
python - "$OUT" <<'PY'
import json, sys, glob, os, csv, collections
for f in sorted(glob.glob(os.path.join(sys.argv[1], "?_?.log"))):
    l = [x for x in open(f) if x.startswith("{")]
    d = json.loads(l[-1]); print(os.path.basename(f), d["value"], d["roofline"]["avg_launch_ms"])
agg = collections.defaultdict(list)
for r in csv.DictReader(open(glob.glob(os.path.join(sys.argv[1], "fetch_b", "*counter_collection.csv"))[0])):
    agg[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    if "volpath" in k: print(k, "FETCH_SIZE GB/launch (x2 gfx950)", 2 * sum(v) / len(v) * 1024 / 1e9)
PY
