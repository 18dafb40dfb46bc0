#!/bin/bash
# round 3: LDS splat table sizes (count / sum slots): W=1 and W=8 training
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03y
mkdir -p $O
for v in base sp1024 sp2048; do
  L=""; [ $v != base ] && L=mitsuba-path-guiding_amd/build_$v/libpgamd.so
  for w in 1 8; do
    PG_LIB=$L PG_TRAIN_ONLY=1 PG_TRAIN_REPS=3 timeout -k 10 200 python -u tools/train_timing.py $w > $O/train_w${w}_$v.log 2>&1 || exit 1
    echo "$v W=$w"; grep "rep 2" $O/train_w${w}_$v.log | sed 's/reset_film.*//'
  done
done
