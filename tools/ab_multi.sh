#!/bin/bash
# A/B/C... of several builds of libpgamd.so on one box, round-robin: tools/ab_multi.sh OUT ROUNDS LIB... -- [bench args]
set -eo pipefail
OUT=$1; ROUNDS=$2; shift 2
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p "$OUT"
for i in $(seq 1 "$ROUNDS"); do
  for k in "${!LIBS[@]}"; do
    PG_LIB=${LIBS[$k]} timeout -k 10 240 python bench.py --no-cpu --no-quality "$@" > "$OUT/v${k}_$i.log" 2>&1
  done
done
python - "$OUT" "${LIBS[@]}" <<'PY'
import json, sys, glob, os
out, libs = sys.argv[1], sys.argv[2:]
for k, lib in enumerate(libs):
    for f in sorted(glob.glob(os.path.join(out, f"v{k}_*.log"))):
        l = [x for x in open(f) if x.startswith("{")]
        if not l: print(f, "no result"); continue
        d = json.loads(l[-1]); kk = d["roofline"].get("kernels", {})
        print(lib, os.path.basename(f), d["value"], {n: v["ms"] for n, v in kk.items()})
PY
