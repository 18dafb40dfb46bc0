#!/bin/bash
# round 5 (ae): strong-scaling rehearsal on one GPU at the checkpoint-3 kernels (tools/shard_timing.py)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05ae
mkdir -p $O
timeout -k 10 500 python -u tools/shard_timing.py > $O/shard_timing.log 2>&1 || { tail -5 $O/shard_timing.log; exit 1; }
tail -8 $O/shard_timing.log
