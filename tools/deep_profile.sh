#!/bin/bash
# Counter passes over the C3 bench (one job + the one-lane calibration pass), one rocprofv3 --pmc run
# per pass (MI355X_MICROARCH.md: never more than the per-block counter limits in one pass).
# usage: tools/deep_profile.sh OUTDIR [extra bench args, e.g. --scene smoke]
set -eo pipefail
OUT=${1:-gpurun_out/deep}
shift || true
EXTRA=("$@")
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d "$OUT/$n" -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu --no-quality "${EXTRA[@]}" > "$OUT/$n.log" 2>&1
}
run sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA
run sq2 SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_LEVEL_WAVES SQ_WAVES GRBM_GUI_ACTIVE
run mem1 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE
run mem2 TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE
echo "deep profile done"
