#!/bin/bash
# round 4 end: C5 rocprofv3 trace + HBM counter passes at HEAD (pmc_volpath_latest.json), then the C5 bench
# line citing them.  usage: PG_REVISION=<hash> tools/r04an_gpu.sh
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04an
mkdir -p $O
timeout -k 10 420 bash tools/profile.sh gpurun_out/prof_r04an_c5 --scene smoke && python tools/pmc_summary.py gpurun_out/prof_r04an_c5 $O/c5 > $O/c5_summary.txt 2>&1 || { echo "c5 profile failed"; exit 1; }
cp $O/pmc_volpath_latest.json profiles/pmc_volpath_latest.json
head -4 $O/c5_summary.txt
timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 1; }
grep "^{" $O/bench_c5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('C5', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('frac_rocprof'), r.get('avg_launch_ms'), r.get('avg_launch_ms_rocprof'), r.get('traffic_over_algorithmic'))"
