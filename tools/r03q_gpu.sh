#!/bin/bash
# round 3: k_volpath refill threshold: identity check, then C5 A/B
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03q
mkdir -p $O
for r in 40 48 56 64; do
  PG_VOL_REFILL=$r timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_refill$r.log 2>&1 || { tail -5 $O/c5_refill$r.log; exit 1; }
done
python - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r03q/c5_*.log")):
    l = [x for x in open(f) if x.startswith("{")]
    if not l: print(f, "no result"); continue
    d = json.loads(l[-1]); r = d["roofline"]
    print(os.path.basename(f), d["value"], d["ms_per_step"], r.get("avg_launch_ms"))
PY
