#!/bin/bash
# round 4: how much of the C5 interaction stage is NEE (shadow walk + transmittance)?  useNee off vs on
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04m
mkdir -p $O
for i in 1 2; do
  for v in nee nonee; do
    P='{}'; [ $v = nonee ] && P='{"useNee": false}'
    timeout -k 10 200 python bench.py --scene smoke --no-cpu --props "$P" > $O/c5_${v}_$i.log 2>&1 || { echo "c5 $v failed"; tail -5 $O/c5_${v}_$i.log; exit 1; }
    grep "^{" $O/c5_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c5 $v', d['value'], d['ms_per_step'], d['segments_per_path'], {k: (v['avg_launch_ms'], v['density_lookups_per_launch']) for k, v in r['kernels'].items()})"
  done
done
