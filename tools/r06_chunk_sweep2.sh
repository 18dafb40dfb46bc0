#!/bin/bash
# Round 6: C3 final-render chunk counts 12 / 15 / 18 / 21 (paths-per-chunk caps 80M / 2^26 / 53M / 46M), interleaved
set -eo pipefail
OUT=${1:-gpurun_out/r06_chunk2}
mkdir -p "$OUT"
for r in 1 2 3; do
  for p in 80000000 67108864 53000000 46000000; do
    timeout -k 10 240 python bench.py --no-cpu --no-quality --steps 5 --warmup 1 --paths-in-flight $p > "$OUT/pif${p}_$r.log" 2>&1
  done
done
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
    l = [x for x in open(f) if x.startswith("{")]
    print(os.path.basename(f), json.loads(l[-1])["value"] if l else "no result")
PY
