#!/bin/bash
# round 5 (f): C5 kernel traces of the round-4 library and this tree's (one job each, --steps 1 --warmup 1)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp
PG_LIB=ab/r04/mitsuba-path-guiding_amd/build/libpgamd.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/r04 -o run --output-format csv -- python3 bench.py --scene smoke --steps 1 --warmup 1 --no-cpu --no-quality > $O/r04.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/r05 -o run --output-format csv -- python3 bench.py --scene smoke --steps 1 --warmup 1 --no-cpu --no-quality > $O/r05.log 2>&1 || exit 1
for v in r04 r05; do echo "== $v"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$O/$v/run_kernel_stats.csv')))
for r in rows[:14]: print(r['Name'][:60].ljust(60), r['Calls'], round(float(r['TotalDurationNs'])/1e6,1), 'ms')
"; done
