#!/bin/bash
# round 5 (ai): counter passes (tools/deep_profile.sh) over C3 and C5 at the checkpoint-3 kernels
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05ai
mkdir -p $O
timeout -k 10 600 bash tools/deep_profile.sh gpurun_out/deep_r05ai_c3 && python tools/deep_summary.py gpurun_out/deep_r05ai_c3 > $O/c3_deep.json || { echo c3 failed; exit 1; }
timeout -k 10 600 bash tools/deep_profile.sh gpurun_out/deep_r05ai_c5 --scene smoke && python tools/deep_summary.py gpurun_out/deep_r05ai_c5 > $O/c5_deep.json || { echo c5 failed; exit 1; }
python - <<'PY'
import json
for n in ("c3", "c5"):
    d = json.load(open(f"gpurun_out/r05ai/{n}_deep.json"))
    for k, v in d.items():
        if v.get("SQ_WAVE_CYCLES", 0) < 1e8: continue
        hit = v["TCC_HIT_sum"] / max(v["TCC_HIT_sum"] + v["TCC_MISS_sum"], 1)
        lat = v["TCP_TCC_READ_REQ_LATENCY_sum"] / max(v["TCP_TCC_READ_REQ_sum"], 1)
        print(n, k, "L2 hit %.3f" % hit, "wait/wave %.3f" % (v["SQ_WAIT_ANY"] / v["SQ_WAVE_CYCLES"]),
              "valu/wave %.3f" % (v["SQ_ACTIVE_INST_VALU"] / v["SQ_WAVE_CYCLES"]), "TCP->TCC latency %.0f" % lat)
PY
