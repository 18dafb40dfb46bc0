#!/bin/bash
# Round 6: path lanes / chunk size re-check with the current kernels (C3 bench, default build)
set -eo pipefail
OUT=${1:-gpurun_out/r06_lanes}
mkdir -p "$OUT"
for r in 1 2; do
  for cfg in "--lanes 3" "--lanes 2" "--lanes 4" "--paths-in-flight 16777216" "--paths-in-flight 67108864"; do
    tag=$(echo "$cfg" | tr -d ' -')
    timeout -k 10 240 python bench.py --no-cpu --no-quality --steps 5 --warmup 1 $cfg > "$OUT/${tag}_$r.log" 2>&1
  done
done
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
    l = [x for x in open(f) if x.startswith("{")]
    print(os.path.basename(f), json.loads(l[-1])["value"] if l else "no result")
PY
