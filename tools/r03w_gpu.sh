#!/bin/bash
# round 3: W=8 training timeline at HEAD (kernel + runtime trace)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03w
mkdir -p $O
export TMPDIR=/tmp
PG_TRAIN_ONLY=1 PG_TRAIN_REPS=4 timeout -k 10 200 rocprofv3 --kernel-trace --runtime-trace -d $O/train_trace -o run --output-format csv -- python3 tools/train_timing.py 8 > $O/train_trace.log 2>&1 || { echo "train trace failed $?"; tail $O/train_trace.log; exit 1; }
python tools/trace_summary.py $O/train_trace --window 20 > $O/train_trace_summary.txt 2>&1; cat $O/train_trace_summary.txt
