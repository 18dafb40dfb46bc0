#!/bin/bash
# A/B/... of bench.py argument sets on one build, round-robin runs:
#   tools/ab_args.sh OUT ROUNDS "ARGS1" "ARGS2" ...
set -eo pipefail
OUT=$1; R=$2; shift 2
mkdir -p "$OUT"
for i in $(seq 1 $R); do
  k=0
  for args in "$@"; do
    timeout -k 10 240 python bench.py --no-cpu --no-quality $args > "$OUT/v${k}_$i.log" 2>&1
    k=$((k + 1))
  done
done
python - "$OUT" "$@" <<'PY'
import json, sys, glob, os
out, sets = sys.argv[1], sys.argv[2:]
for k, a in enumerate(sets):
    for f in sorted(glob.glob(os.path.join(out, f"v{k}_*.log"))):
        l = [x for x in open(f) if x.startswith("{")]
        if not l: print(repr(a), os.path.basename(f), "no result"); continue
        d = json.loads(l[-1])
        print(repr(a), os.path.basename(f), d["value"], d["ms_per_step"], d["segments_per_path"])
PY
