#!/bin/bash
# Round 6: the auto chunk policy (12 chunks for C3's final render) against fixed 2^26 and 2^25 caps, interleaved
set -eo pipefail
OUT=${1:-gpurun_out/r06_chunk3}
mkdir -p "$OUT"
for r in 1 2 3; do
  for p in 0 67108864 33554432; do
    timeout -k 10 240 python bench.py --no-cpu --no-quality --steps 5 --warmup 1 --paths-in-flight $p > "$OUT/pif${p}_$r.log" 2>&1
  done
done
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
    l = [x for x in open(f) if x.startswith("{")]
    print(os.path.basename(f), json.loads(l[-1])["value"] if l else "no result")
PY
