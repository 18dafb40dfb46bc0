#!/bin/bash
# Round 6: BVH build constants with the paired leaf tests (env knobs of pg_bvh.cpp, no rebuild):
# triangle-test cost 1 (default) / 0.7 / 0.5 and the never-split leaf size 2 (default) / 3 / 4, interleaved
set -eo pipefail
OUT=${1:-gpurun_out/r06_bvh}
mkdir -p "$OUT"
for r in 1 2; do
  for cfg in "1 2" "0.7 2" "0.5 2" "1 3" "1 4"; do
    set -- $cfg
    PG_BVH_TRI_COST=$1 PG_BVH_LEAF_TARGET=$2 timeout -k 10 240 python bench.py --no-cpu --no-quality --steps 5 --warmup 1 > "$OUT/tc$1_lt$2_$r.log" 2>&1
  done
done
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
    l = [x for x in open(f) if x.startswith("{")]
    if not l: print(os.path.basename(f), "no result"); continue
    d = json.loads(l[-1]); k = d["roofline"]["kernels"]
    print(os.path.basename(f), d["value"], {n: v["ms"] for n, v in k.items()})
PY
