#!/bin/bash
# round 3: k_volpath one interaction kind per iteration (PG_VOL_SURF_WAIT): identity test, C5 A/B
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_volume.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; s=$?; tail -4 $O/tests.log; [ $s -eq 0 ] || exit 1
for w in 0 1 2 4 8; do
  PG_VOL_SURF_WAIT=$w timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_wait$w.log 2>&1 || { tail -5 $O/c5_wait$w.log; exit 1; }
done
python - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r03u/c5_*.log")):
    l = [x for x in open(f) if x.startswith("{")]
    if not l: print(f, "no result"); continue
    d = json.loads(l[-1]); r = d["roofline"]
    print(os.path.basename(f), d["value"], d["ms_per_step"], r.get("avg_launch_ms"))
PY
