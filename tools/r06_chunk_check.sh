#!/bin/bash
# Round 6: the auto chunk size (2^26 for C3's final render) — config tests, then the default bench twice
set -eo pipefail
OUT=${1:-gpurun_out/r06_chunk_check}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_tail.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
for r in 1 2; do
  timeout -k 10 240 python bench.py --no-cpu --no-quality --steps 5 --warmup 1 > "$OUT/bench_$r.log" 2>&1
done
grep -h '^{' "$OUT"/bench_*.log | python -c "import sys, json; [print(json.loads(l)['value']) for l in sys.stdin]"
