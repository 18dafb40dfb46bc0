#!/bin/bash
# tools-style env A/B: OUT ROUNDS VAR -- bench args; alternates runs without / with VAR=1
set -eo pipefail
OUT=$1; R=$2; VAR=$3; shift 3; [ "$1" == "--" ] && shift
mkdir -p "$OUT"
for i in $(seq 1 $R); do
  timeout -k 10 240 python bench.py --no-cpu --no-quality "$@" > "$OUT/off_$i.log" 2>&1
  env $VAR=1 timeout -k 10 240 python bench.py --no-cpu --no-quality "$@" > "$OUT/on_$i.log" 2>&1
done
for f in "$OUT"/*.log; do python - "$f" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")]
d = json.loads(l[-1]); k = d["roofline"].get("kernels", {})
print(sys.argv[1].split("/")[-1], d["value"], {n: v["ms"] for n, v in k.items()})
PY
done
