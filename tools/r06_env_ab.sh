#!/bin/bash
# A/B of a run-time switch on one box, alternating runs: tools/r06_env_ab.sh OUT "VAR=a" "VAR=b" [bench args]
set -eo pipefail
OUT=$1; A=$2; B=$3; shift 3
mkdir -p "$OUT"
for i in 1 2; do
  env $A timeout -k 10 240 python bench.py --no-cpu --no-quality "$@" > "$OUT/a_$i.log" 2>&1
  env $B timeout -k 10 240 python bench.py --no-cpu --no-quality "$@" > "$OUT/b_$i.log" 2>&1
done
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*_?.log"))):
    l = [x for x in open(f) if x.startswith("{")]
    if not l: print(f, "no result"); continue
    d = json.loads(l[-1]); k = d["roofline"].get("kernels", {})
    print(os.path.basename(f), d["value"], d["ms_per_step"], {n: v["ms"] for n, v in k.items()})
PY
