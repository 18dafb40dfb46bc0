#!/bin/bash
# A/B of the XCD-banded camera shard map (PG_CAMERA_BANDS = bands of the local pixels; 0 = interleaved map) on
# C3: bench lines with the calibration's per-kernel launch averages, alternating, same box
set -o pipefail
out=${1:-gpurun_out/r06e}
mkdir -p $out
for i in 1 2; do
  for b in ${BANDS:-0 64 512}; do
    PG_CAMERA_BANDS=$b timeout -k 10 240 python3 bench.py --steps 5 --warmup 1 --no-cpu --no-quality \
      > $out/bands${b}_$i.json 2> $out/bands${b}_$i.err || exit 1
    python3 -c "import json;d=json.load(open('$out/bands${b}_$i.json'));r=d['roofline'];print('bands=$b run $i', d['value'], {k:v['avg_launch_ms'] for k,v in r['kernels'].items()})"
  done
done
