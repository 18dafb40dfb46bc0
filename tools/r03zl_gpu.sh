#!/bin/bash
# round 3 final: strong-scaling rehearsal on one GPU (rank 0's shard of the C3 job at W = 1/2/4/8)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r03zl
mkdir -p $O
timeout -k 10 400 python -u tools/shard_timing.py 1,2,4,8 > $O/shard_timing.log 2>&1 || { tail -5 $O/shard_timing.log; exit 1; }
cat $O/shard_timing.log
