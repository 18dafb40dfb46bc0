#!/bin/bash
# A/B of two builds of libpgamd.so on one box, alternating runs: tools/ab_bench.sh OUT LIB_A LIB_B [bench args]
set -eo pipefail
OUT=$1; A=$2; B=$3; shift 3
mkdir -p "$OUT"
for i in 1 2; do
  PG_LIB=$A timeout -k 10 240 python bench.py --no-cpu --no-quality "$@" > "$OUT/a_$i.log" 2>&1
  PG_LIB=$B timeout -k 10 240 python bench.py --no-cpu --no-quality "$@" > "$OUT/b_$i.log" 2>&1
done
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*_?.log"))):
    l = [x for x in open(f) if x.startswith("{")]
    if not l: print(f, "no result"); continue
    d = json.loads(l[-1]); k = d["roofline"].get("kernels", {})
    print(os.path.basename(f), d["value"], d["ms_per_step"], d["segments_per_path"],
          {n: v["ms"] for n, v in k.items()})
PY
