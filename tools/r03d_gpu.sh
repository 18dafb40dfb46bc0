#!/bin/bash
# round 3: learned-fraction debug, C3 quality per fraction mode, GPU suite, ray-sort A/B
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r03d
timeout -k 10 120 python -u tools/dbg_learned.py > gpurun_out/r03d/dbg_learned.log 2>&1; cat gpurun_out/r03d/dbg_learned.log | tail -20
for m in learned albedo fixed; do
  timeout -k 10 300 python -u tools/quality_c3.py --gt tests/golden/c3_gt.npz --props "{\"bsdfSamplingFractionBound\": \"$m\"}" > gpurun_out/r03d/q_$m.log 2>&1 || { echo "quality $m failed"; tail -20 gpurun_out/r03d/q_$m.log; exit 1; }
  tail -1 gpurun_out/r03d/q_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['guided_vs_unguided'], d['guided_discard']['relmse_exposed'], d['guided_discard']['relmse_exposed_trim999'], d['unguided_equal_spp']['relmse_exposed'], d['guided_discard']['seconds'])"
done
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r03d/gpu_tests.log 2>&1; tail -5 gpurun_out/r03d/gpu_tests.log
for i in 1 2; do
  timeout -k 10 240 python bench.py --no-cpu --no-quality > gpurun_out/r03d/sort0_$i.log 2>&1 || exit 1
  PG_RAY_SORT=1 timeout -k 10 240 python bench.py --no-cpu --no-quality > gpurun_out/r03d/sort1_$i.log 2>&1 || exit 1
done
python - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r03d/sort*.log")):
    l = [x for x in open(f) if x.startswith("{")]
    if not l: print(f, "no result"); continue
    d = json.loads(l[-1]); k = d["roofline"].get("kernels", {})
    print(os.path.basename(f), d["value"], d["ms_per_step"], {n: v["ms"] for n, v in k.items()})
PY
