"""GPU busy fraction and per-kernel time from a rocprofv3 kernel-trace CSV (development helper).
usage: busy.py run_kernel_trace.csv"""
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
t0, t1 = iv[0][0], max(e for _, e, _ in iv)
busy, cur_s, cur_e = 0, None, None
for s, e, _ in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None: busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"span {(t1-t0)/1e6:.1f} ms  busy(union) {busy/1e6:.1f} ms  ({busy/(t1-t0):.3f})")
tot = collections.Counter(); cnt = collections.Counter()
for s, e, n in iv:
    k = n.split("(")[0].split("<")[0] if "k_shade" not in n else n.split("(")[0]
    tot[k] += e - s; cnt[k] += 1
for k, v in tot.most_common(12):
    print(f"{k[:60]:60s} {cnt[k]:7d} {v/1e6:10.1f} ms  avg {v/cnt[k]/1e3:8.1f} us")
# largest idle gaps and the kernels around them
gaps = []
prev_e, prev_n = None, None
for s, e, n in iv:
    if prev_e is not None and s > prev_e:
        gaps.append((s - prev_e, prev_n.split("(")[0], n.split("(")[0], (prev_e - t0) / 1e6))
    if prev_e is None or e > prev_e:
        prev_e, prev_n = e, n
gaps.sort(reverse=True)
tot_gap = sum(g[0] for g in gaps)
print(f"gaps: {len(gaps)} total {tot_gap/1e6:.1f} ms; >1ms: {sum(g[0] for g in gaps if g[0] > 1e6)/1e6:.1f} ms")
for g in gaps[:12]:
    print(f"  {g[0]/1e6:8.2f} ms at {g[3]:9.1f} ms  after {g[1][:30]:30s} before {g[2][:30]}")
