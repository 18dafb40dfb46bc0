#!/bin/bash
# round 3: W=8 training timeline (kernel + runtime trace), then HEAD profiles of C3 and C5
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03f
mkdir -p $O
export TMPDIR=/tmp
PG_TRAIN_ONLY=1 PG_TRAIN_REPS=4 PG_DEBUG_REFIT=1 timeout -k 10 200 rocprofv3 --kernel-trace --runtime-trace -d $O/train_trace -o run --output-format csv -- python3 tools/train_timing.py 8 > $O/train_trace.log 2>&1 || { echo "train trace failed $?"; tail $O/train_trace.log; exit 1; }
python tools/trace_summary.py $O/train_trace --window 45 > $O/train_trace_summary.txt 2>&1; cat $O/train_trace_summary.txt
bash tools/profile.sh gpurun_out/prof_r03f && bash tools/profile.sh gpurun_out/prof_r03f_c5 --scene smoke && echo profiles ok
