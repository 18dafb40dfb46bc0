#!/bin/bash
# round 4 final checkpoint: rocprofv3 kernel traces + HBM counter passes of C3 and C5 (their summaries
# become profiles/pmc_latest.json / pmc_volpath_latest.json, which the bench lines cite), then the GPU
# suite, smoke() and both bench lines at this revision.  usage: PG_REVISION=<hash> tools/r04z_gpu.sh
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${CHECKPOINT:-r04z}
mkdir -p $O
timeout -k 10 420 bash tools/profile.sh gpurun_out/prof_${CHECKPOINT:-r04z}_c3 && python tools/pmc_summary.py gpurun_out/prof_${CHECKPOINT:-r04z}_c3 $O/c3 > $O/c3_summary.txt 2>&1 || { echo "c3 profile failed"; exit 1; }
cp $O/pmc_latest.json profiles/pmc_latest.json
timeout -k 10 420 bash tools/profile.sh gpurun_out/prof_${CHECKPOINT:-r04z}_c5 --scene smoke && python tools/pmc_summary.py gpurun_out/prof_${CHECKPOINT:-r04z}_c5 $O/c5 > $O/c5_summary.txt 2>&1 || { echo "c5 profile failed"; exit 1; }
cp $O/pmc_volpath_latest.json profiles/pmc_volpath_latest.json
head -8 $O/c3_summary.txt $O/c5_summary.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1; s=$?; grep -E "passed|failed|FAILED" $O/gpu_tests.log | head; [ $s -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 1; }
timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 1; }
for f in $O/bench_c3.log $O/bench_c5.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('frac_rocprof'))"; done
