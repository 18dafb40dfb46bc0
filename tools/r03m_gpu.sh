#!/bin/bash
# round 3: C5 A/B: previous build, + cached S-tree leaf box in guided free flight, + corner-packed density; volume GPU tests first
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03m
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal status $1 in $2"; exit 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_volume.py tests/test_gpu_bidir_pin.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; s=$?; tail -4 $O/tests.log; fatal $s tests
[ $s -eq 0 ] || exit 1
for i in 1 2; do
  PG_LIB=mitsuba-path-guiding_amd/build_base/libpgamd.so timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_base_$i.log 2>&1 || { tail -5 $O/c5_base_$i.log; exit 1; }
  PG_LIB=mitsuba-path-guiding_amd/build_box/libpgamd.so timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_box_$i.log 2>&1 || { tail -5 $O/c5_box_$i.log; exit 1; }
  timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/c5_corners_$i.log 2>&1 || { tail -5 $O/c5_corners_$i.log; exit 1; }
done
python - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r03m/c5_*.log")):
    l = [x for x in open(f) if x.startswith("{")]
    if not l: print(f, "no result"); continue
    d = json.loads(l[-1]); r = d["roofline"]
    print(os.path.basename(f), d["value"], d["ms_per_step"], r.get("avg_launch_ms"), r.get("density_lookups_per_launch"))
PY
