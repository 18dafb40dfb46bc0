set -eo pipefail
mkdir -p gpurun_out/ab_gmat
tools/ab_bench.sh gpurun_out/ab_gmat/c3 mitsuba-path-guiding_amd/build/libpgamd.so ab/old/libpgamd.so --steps 3 --warmup 1
for L in mitsuba-path-guiding_amd/build/libpgamd.so ab/old/libpgamd.so; do
  PG_LIB=$L timeout -k 10 200 python bench.py --scene smoke --steps 2 --warmup 1 --no-cpu > gpurun_out/ab_gmat/c5_$(basename $(dirname $(dirname $L))).log 2>&1
done
grep -h '"value"' gpurun_out/ab_gmat/c5_*.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('C5', d['value'], d['roofline']['avg_launch_ms'])"
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/ab_gmat/c5w -o run --output-format csv -- python3 bench.py --scene smoke --steps 1 --warmup 0 --no-cpu > gpurun_out/ab_gmat/c5w.log 2>&1
echo done
