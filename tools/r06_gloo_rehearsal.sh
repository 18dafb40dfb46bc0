#!/bin/bash
# Round 6: the driver's multi-GPU bench command (torch.distributed.run, one rank per GPU) rehearsed on one GPU with
# PG_DIST_BACKEND=gloo (ranks share the device; RCCL refuses that), at 2, 4 and 8 ranks: launcher, per-rank start-up
# report, deadlines, tile shard, statistics exchange, max-over-ranks timing and the rank-0 line of the current bench.py
set -eo pipefail
OUT=${1:-gpurun_out/r06_gloo}
mkdir -p "$OUT"
export PG_DIST_BACKEND=gloo
for n in 2 4 8; do
  echo "ranks $n"
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --steps 3 --warmup 1 > "$OUT/gloo$n.log" 2>&1
  grep '^{' "$OUT/gloo$n.log" | tail -1 | cut -c1-400
done
