#!/bin/bash
# round 3: W=8 training timeline at HEAD (kernel + runtime trace)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03w
mkdir -p $O
export TMPDIR=/tmp
PG_TRAIN_ONLY=1 PG_TRAIN_REPS=4 timeout -k 10 200 rocprofv3 --kernel-trace --runtime-trace -d $O/train_trace -o run --output-format csv -- python3 tools/train_timing.py 8 > $O/train_trace.log 2>&1 || { echo "train trace failed $?"; tail $O/train_trace.log; exit 1; }
python tools/trace_summary.py $O/train_trace --window 20 > $O/train_trace_summary.txt 2>&1; cat $O/train_trace_summary.txt
for t in 131072 1048576 4194304; do
  PG_TAIL_PATHS=$t PG_TRAIN_ONLY=1 PG_TRAIN_REPS=3 timeout -k 10 200 python -u tools/train_timing.py 8 > $O/train_w8_tail$t.log 2>&1 || exit 1
  echo "W=8 tail=$t"; grep "rep 2" $O/train_w8_tail$t.log
  PG_TAIL_PATHS=$t PG_TRAIN_ONLY=1 PG_TRAIN_REPS=3 timeout -k 10 200 python -u tools/train_timing.py 1 > $O/train_w1_tail$t.log 2>&1 || exit 1
  echo "W=1 tail=$t"; grep "rep 2" $O/train_w1_tail$t.log
done
