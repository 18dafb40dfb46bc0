"""HIP-event vs rocprofv3 kernel durations of bench.py's calibration context.

usage: python tools/reconcile.py TRACE_DIR BENCH_LOG [BENCH_LOG ...]
TRACE_DIR: a rocprofv3 --kernel-trace output (run_kernel_trace.csv) of a bench.py run; the BENCH_LOGs are
bench.py outputs (the first one printed under that trace, the others plain runs for comparison).  Prints,
per path kernel, the calibration stream's average launch duration in the trace against every log's
`roofline.kernels[k].avg_launch_ms`.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import base_name, calibration_stream, rows_of  # noqa: E402


def main(trace_dir, logs):
    rows = rows_of(os.path.join(trace_dir, "run_kernel_trace.csv"))
    cal = calibration_stream(rows)
    acc = {}
    for r in rows:
        if r.get("Stream_Id") != cal:
            continue
        k = base_name(r["Kernel_Name"])
        a = acc.setdefault(k, [])
        a.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    lines = []
    for f in logs:
        l = [x for x in open(f) if x.startswith("{")]
        lines.append((f, json.loads(l[-1]) if l else None))
    for k, v in sorted(acc.items()):
        if len(v) < 2:
            continue
        s = f"{k:14s} rocprof {len(v):3d} launches avg {sum(v) / len(v) / 1e6:.4f} ms"
        for f, d in lines:
            e = (d or {}).get("roofline", {}).get("kernels", {}).get(k)
            if e:
                s += f" | {os.path.basename(f)} {e['launches']} x {e['avg_launch_ms']:.4f} ms"
        print(s)
    for f, d in lines:
        if d:
            print(os.path.basename(f), "value", d["value"], "ms_per_step", d["ms_per_step"])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
