#!/bin/bash
# round 3: C5 majorant-cell A/B (8 default, 4, 16) then counter passes over the C5 bench
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03k
mkdir -p $O
for i in 1 2; do
  for c in 8 4 16; do
    L=""; [ $c != 8 ] && L=mitsuba-path-guiding_amd/build_cell$c/libpgamd.so
    PG_LIB=$L timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_cell${c}_$i.log 2>&1 || { echo "bench cell $c failed"; tail -5 $O/c5_cell${c}_$i.log; exit 1; }
  done
done
python - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r03k/c5_*.log")):
    l = [x for x in open(f) if x.startswith("{")]
    if not l: print(f, "no result"); continue
    d = json.loads(l[-1]); r = d["roofline"]
    print(os.path.basename(f), d["value"], d["ms_per_step"], r.get("avg_launch_ms"), r.get("density_lookups_per_launch"))
PY
bash tools/deep_profile.sh gpurun_out/deep_r03k_c5 --scene smoke && python tools/deep_summary.py gpurun_out/deep_r03k_c5 > gpurun_out/deep_r03k_c5/summary.json && echo deep ok
