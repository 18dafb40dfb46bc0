"""Timeline summary of a rocprofv3 --kernel-trace --runtime-trace run (development helper): for the
last `--window` ms of the trace, the kernels and HIP API calls by total time, and the GPU-idle gaps.

usage: python tools/trace_summary.py <rocprofv3 output dir> [--window MS] [--start-after-kernel NAME]"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def col(r, *names):
    for n in names:
        if n in r:
            return r[n]
    raise KeyError(names)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--window", type=float, default=250.0, help="ms at the end of the trace")
    ap.add_argument("--skip-last-kernel", default="", help="end the window before the last launch of this kernel")
    a = ap.parse_args()
    ks = rows(os.path.join(a.dir, "**", "*kernel_trace.csv"))
    api = rows(os.path.join(a.dir, "**", "*hip_api_trace.csv"))
    K = sorted(((int(col(r, "Start_Timestamp")), int(col(r, "End_Timestamp")), col(r, "Kernel_Name")) for r in ks))
    A = sorted(((int(col(r, "Start_Timestamp")), int(col(r, "End_Timestamp")), col(r, "Function")) for r in api))
    end = K[-1][1]
    if a.skip_last_kernel:
        last = [k for k in K if a.skip_last_kernel in k[2]]
        if last:
            end = last[-1][0]
    t0 = end - int(a.window * 1e6)
    Kw = [k for k in K if k[0] >= t0 and k[1] <= end]
    Aw = [x for x in A if x[0] >= t0 and x[1] <= end]
    busy = defaultdict(lambda: [0, 0])
    for s, e, n in Kw:
        n = n.split("(")[0].replace("void ", "")[:40]
        busy[n][0] += 1
        busy[n][1] += e - s
    print(f"window {a.window} ms ending {end}: {len(Kw)} kernels, {len(Aw)} API calls")
    for n, (c, t) in sorted(busy.items(), key=lambda x: -x[1][1]):
        print(f"  kernel {n:42s} {c:6d} calls {t / 1e6:8.3f} ms")
    api_t = defaultdict(lambda: [0, 0])
    for s, e, n in Aw:
        api_t[n][0] += 1
        api_t[n][1] += e - s
    for n, (c, t) in sorted(api_t.items(), key=lambda x: -x[1][1])[:15]:
        print(f"  api    {n:42s} {c:6d} calls {t / 1e6:8.3f} ms")
    # GPU idle: union of kernel intervals
    idle, cur = 0, t0
    gaps = []
    for s, e, n in Kw:
        if s > cur:
            idle += s - cur
            gaps.append((s - cur, cur, n))
        cur = max(cur, e)
    idle += max(0, end - cur)
    print(f"  GPU idle {idle / 1e6:.3f} ms of {a.window} ms; largest gaps (us, before kernel):")
    for g, s, n in sorted(gaps, reverse=True)[:12]:
        print(f"    {g / 1e3:9.1f} us at {(s - t0) / 1e6:8.3f} ms before {n.split('(')[0][:40]}")


if __name__ == "__main__":
    main()
