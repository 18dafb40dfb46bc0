#!/bin/bash
# round 4: replay the diverging C3 paths with the PG_WATCH vertex log (GPU vs oracle, field by field)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 700 python -u tools/diverge_c3.py $O/diverge.json --top 8 > $O/diverge.log 2>&1 || { tail -5 $O/diverge.log; exit 1; }
cut -c1-1500 $O/diverge.log | head -60
