#!/bin/bash
# round 5 (b): FETCH_SIZE calibration of the gather widths (tools/fetch_calib.hip), then the HIP-event vs
# rocprofv3 duration reconciliation of the bench's calibration context (plain run, the same command under
# --kernel-trace, and the profile.sh form --steps 1 --warmup 0)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05b
mkdir -p $O/cal
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || echo "counter list failed"
timeout -k 10 120 tools/fetch_calib > $O/cal/cases.jsonl || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/cal/fetch -o run --output-format csv -- tools/fetch_calib > $O/cal/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum -d $O/cal/req -o run --output-format csv -- tools/fetch_calib > $O/cal/req.log 2>&1 || exit 1
python tools/fetch_calib_summary.py $O/cal $O/fetch_calib.json
timeout -k 10 300 python bench.py --no-cpu --no-quality > $O/rec_plain.log 2>&1 || exit 1
timeout -k 10 420 rocprofv3 --kernel-trace --stats -T -d $O/rec_trace -o run --output-format csv -- python3 bench.py --no-cpu --no-quality > $O/rec_traced.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu --no-quality > $O/rec_cold.log 2>&1 || exit 1
python tools/reconcile.py $O/rec_trace $O/rec_traced.log $O/rec_plain.log $O/rec_cold.log
