#!/bin/bash
# round 3: k_volpath refill threshold: identity check, then C5 A/B
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 200 python -u tools/vol_refill_check.py > $O/refill_check.log 2>&1; s=$?; cat $O/refill_check.log | tail -5; [ $s -eq 0 ] || exit 1
for r in 1 16 32 8; do
  PG_VOL_REFILL=$r timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_refill$r.log 2>&1 || { tail -5 $O/c5_refill$r.log; exit 1; }
done
python - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r03p/c5_*.log")):
    l = [x for x in open(f) if x.startswith("{")]
    if not l: print(f, "no result"); continue
    d = json.loads(l[-1]); r = d["roofline"]
    print(os.path.basename(f), d["value"], d["ms_per_step"], r.get("avg_launch_ms"))
PY
