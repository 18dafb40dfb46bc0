#!/bin/bash
# Round 6: chunk counts for an N-GPU rank's share of C3's final render, emulated on one GPU with a smaller spp:
# spp 128 (N = 8: default 6 chunks, 9, 12) and spp 256 (N = 4: default 9 chunks, 12), interleaved
set -eo pipefail
OUT=${1:-gpurun_out/r06_shard_chunks}
mkdir -p "$OUT"
for r in 1 2 3; do
  for cfg in "128 0" "128 13824000" "128 10137600" "256 0" "256 20275200"; do
    set -- $cfg
    timeout -k 10 240 python bench.py --no-cpu --no-quality --steps 5 --warmup 1 --spp $1 --paths-in-flight $2 > "$OUT/spp$1_pif$2_$r.log" 2>&1
  done
done
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
    l = [x for x in open(f) if x.startswith("{")]
    print(os.path.basename(f), json.loads(l[-1])["value"] if l else "no result")
PY
