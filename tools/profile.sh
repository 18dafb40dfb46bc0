#!/bin/bash
# rocprofv3 evidence for bench.py: kernel trace + stats (timed config), then separate PMC passes
# for FETCH_SIZE and WRITE_SIZE (MI355X_MICROARCH.md §HBM: never combined with other tracing).
# usage: tools/profile.sh OUTDIR [extra bench args, e.g. --scene smoke]
set -eo pipefail
OUT=${1:-gpurun_out/prof}
shift || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --no-quality "$@" > "$OUT/trace.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/fetch" -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --no-quality "$@" > "$OUT/fetch.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/write" -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --no-quality "$@" > "$OUT/write.log" 2>&1
echo "profile done"
