#!/bin/bash
# round 5 (c): memory-side read latency (TCC_EA0_RDREQ_LEVEL / RDREQ) of the calibration gathers (Infinity
# Cache vs HBM) and of the C3 bench's calibration launches (k_rays split), then C5 A/B of the deferred
# transmittance walks: own stage overlapped with the next flights (default), own stage in line on the lane
# stream, inline in k_vvertex
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05c
mkdir -p $O/cal
export TMPDIR=/tmp
timeout -k 10 120 tools/fetch_calib > $O/cal/cases.jsonl || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum -d $O/cal/lat -o run --output-format csv -- tools/fetch_calib > $O/cal/lat.log 2>&1 || exit 1
python tools/fetch_calib_summary.py $O/cal $O/fetch_calib_latency.json
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum -d $O/c3lat -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-quality > $O/c3lat.log 2>&1 || exit 1
python tools/ea_latency.py $O/c3lat 12
for i in 1 2; do
  timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_overlap_$i.log 2>&1 || exit 1
  PG_VOL_NEE_OVERLAP=0 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_stage_$i.log 2>&1 || exit 1
  PG_VOL_NEE_STAGE=0 timeout -k 10 240 python bench.py --scene smoke --no-cpu --no-quality > $O/c5_inline_$i.log 2>&1 || exit 1
done
for f in $O/c5_*.log; do grep "^{" $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], {n: v.get('ms') for n, v in r.get('kernels', {}).items()})"; done
