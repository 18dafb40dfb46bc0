#!/bin/bash
# rocprofv3 evidence for bench.py: kernel trace + stats (the bench's default steps / warmup, so the calibration
# launches run on a GPU as warm as in the driver's line: round 5, profiles/r05b_fetch_calib/reconcile.txt),
# then separate PMC passes (one job each)
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
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-quality "$@" > "$OUT/trace.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/fetch" -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --no-quality "$@" > "$OUT/fetch.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/write" -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu --no-quality "$@" > "$OUT/write.log" 2>&1
echo "profile done"
