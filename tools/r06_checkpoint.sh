#!/bin/bash
# Round-6 checkpoint, one gpurun call: GPU suite, smoke(), rocprofv3 trace + HBM counter passes of C3 and C5 (their
# summaries become this box's profiles/pmc_latest.json / pmc_volpath_latest.json before the bench lines run, so
# the lines' headline fractions come from the same box and revision), then both bench lines with CPU baselines.
# usage: PG_REVISION=<git head> tools/r06_checkpoint.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/r06_ckpt}
cd "$(dirname "$0")/.."
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "gpu suite" && timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 &&
echo "smoke" && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
echo "profile c3" && tools/profile.sh "$OUT/prof_c3" &&
python tools/pmc_summary.py "$OUT/prof_c3" "$OUT/c3" > "$OUT/c3_pmc_summary.txt" &&
echo "profile c5" && tools/profile.sh "$OUT/prof_c5" --scene smoke &&
python tools/pmc_summary.py "$OUT/prof_c5" "$OUT/c5" > "$OUT/c5_pmc_summary.txt" &&
cp "$OUT/pmc_latest.json" profiles/pmc_latest.json && cp "$OUT/pmc_volpath_latest.json" profiles/pmc_volpath_latest.json &&
echo "bench c3" && timeout -k 10 600 python bench.py > "$OUT/bench_c3.log" 2>&1 &&
echo "bench c5" && timeout -k 10 600 python bench.py --scene smoke > "$OUT/bench_c5.log" 2>&1 &&
echo "checkpoint done"
