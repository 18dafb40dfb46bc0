#!/bin/bash
# SQ (shader sequencer) counters per kernel for the bench workload: where the waves spend cycles.
# usage: tools/sq_profile.sh OUTDIR [bench args]
set -eo pipefail
OUT=${1:-gpurun_out/sq}
shift || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
    SQ_INSTS_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU -d "$OUT/sq" -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu "$@" > "$OUT/sq.log" 2>&1
echo "sq done"
