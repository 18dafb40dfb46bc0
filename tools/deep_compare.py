"""Per-kernel ratios of two tools/deep_summary.py outputs (e.g. round 5's and round 6's C3 counters):
L2 hit rate, share of wave cycles waiting, mean L1->L2 read latency (cycles), VALU wave-instructions per launch.
usage: python tools/deep_compare.py A.json B.json [kernel ...]"""
import json
import sys


def ratios(k):
    n = max(k.get("calls", 0), 1)
    hit, miss = k.get("TCC_HIT_sum", 0.0), k.get("TCC_MISS_sum", 0.0)
    req = k.get("TCP_TCC_READ_REQ_sum", 0.0)
    return {
        "l2_hit": round(hit / (hit + miss), 3) if hit + miss else None,
        "wait_share": round(k["SQ_WAIT_ANY"] / k["SQ_WAVE_CYCLES"], 3) if k.get("SQ_WAVE_CYCLES") else None,
        "l1_l2_read_latency_cycles": round(k["TCP_TCC_READ_REQ_LATENCY_sum"] / req, 1) if req else None,
        "valu_insts_per_launch": round(k.get("SQ_INSTS_VALU", 0.0) / n / 1e6, 2),
        "vmem_rd_insts_per_launch": round(k.get("SQ_INSTS_VMEM_RD", 0.0) / n / 1e6, 3),
        "launches": k.get("calls", 0),
    }


a, b = json.load(open(sys.argv[1])), json.load(open(sys.argv[2]))
names = sys.argv[3:] or ["k_trace", "k_shade_all", "k_rays"]
print(json.dumps({n: {"a": ratios(a[n]), "b": ratios(b[n])} for n in names if n in a and n in b}, indent=1))
