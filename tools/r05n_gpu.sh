#!/bin/bash
# round 5 (n): material table staged in LDS per shading block (build_ldsmat: SHADE_LDS_MATS=64) against the
# default, C3, alternating; then the C3 profile (trace at the bench's own steps) and a bench line in one call
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05n
mkdir -p $O
L=mitsuba-path-guiding_amd
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_default_$i.log 2>&1 || exit 1
  PG_LIB=$L/build_ldsmat/libpgamd.so timeout -k 10 240 python bench.py --no-cpu --no-quality > $O/c3_ldsmat_$i.log 2>&1 || exit 1
done
for f in $O/c3_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], {n: v.get('ms') for n, v in r.get('kernels', {}).items()})"; done
echo "c3 profile"
timeout -k 10 600 bash tools/profile.sh gpurun_out/prof_r05n_c3 && python tools/pmc_summary.py gpurun_out/prof_r05n_c3 $O/c3 > $O/c3_summary.txt 2>&1 || { echo "c3 profile failed"; exit 1; }
head -4 $O/c3_summary.txt
cp $O/pmc_latest.json profiles/pmc_latest.json
timeout -k 10 300 python bench.py --no-cpu --no-quality > $O/bench_c3_after_profile.log 2>&1 || exit 1
grep "^{" $O/bench_c3_after_profile.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('line', d['value'], r['frac'], r.get('frac_rocprof'), r.get('avg_launch_ms'), r.get('avg_launch_ms_rocprof'))"
