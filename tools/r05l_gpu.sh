#!/bin/bash
# round 5 (l): the guided C3 job's phases against the unguided render (tools/guided_overhead.py)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 400 python tools/guided_overhead.py 3 > $O/guided_overhead.log 2>&1 || { tail -5 $O/guided_overhead.log; exit 1; }
tail -4 $O/guided_overhead.log
