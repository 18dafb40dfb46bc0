#!/bin/bash
# round 4: C5 index-check build (16^3 majorant cells, the round-3 fault configuration) on the full C5
# job, then the product C5 bench and the volume GPU tests with the emitter re-walk guard
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 400 python -u tools/volcheck_c5.py 2 > $O/volcheck.log 2>&1; s=$?; tail -4 $O/volcheck.log; [ $s -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --scene smoke --no-cpu > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 1; }
grep "^{" $O/bench_c5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 400 python -u -m pytest tests/test_gpu_volume.py tests/test_gpu_bidir_pin.py -x -q --timeout 200 --timeout-method thread > $O/gpu_vol_tests.log 2>&1; s=$?; tail -3 $O/gpu_vol_tests.log; [ $s -eq 0 ] || exit 1
# lane utilisation of k_volpath (divergence: the case for a volumetric wavefront)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
grep -i -E "VALUUtil|THREAD_CYCLES_VALU|SQ_INSTS_VALU" $O/avail.txt | head -20 || true
timeout -s KILL 240 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace -d $O/pmc_valu -o run -- python bench.py --scene smoke --no-cpu --steps 1 --warmup 0 > $O/pmc_valu.log 2>&1 || { echo "pmc pass failed"; tail -5 $O/pmc_valu.log; }
