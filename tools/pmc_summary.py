"""Summarise a tools/profile.sh output directory into profiles/.

Per kernel: calls, average duration (kernel trace), and HBM traffic per launch from the separate
FETCH_SIZE / WRITE_SIZE passes.  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts
64-B units for 128-B requests, i.e. half the bytes of wide (16 B/lane) reads -> doubled here;
WRITE_SIZE is taken as-is.  Both counters are in KiB.
usage: python tools/pmc_summary.py gpurun_out/prof_rNN profiles/rNN
"""
import csv
import json
import os
import sys
from collections import defaultdict


def load_counter(path, name):
    acc = defaultdict(list)
    if not os.path.exists(path):
        return {}
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != name:
            continue
        acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(src, dst_prefix):
    stats = {}
    for row in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        stats[row["Name"]] = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"]),
                              "total_ns": float(row["TotalDurationNs"]), "pct": float(row["Percentage"])}
    fetch = load_counter(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = load_counter(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    out = {"source": src, "correction": "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per launch", "kernels": {}}
    names = {"k_trace": "pg_trace_closest", "k_shade": "pg_shade", "k_shadow": "pg_trace_shadow",
             "k_splat": "pg_splat", "k_commit": "pg_commit", "k_film": "pg_film", "k_camera": "pg_camera"}
    for k, s in stats.items():
        key = names.get(k, k)
        e = dict(s)
        if k in fetch or k in write:
            f, w = fetch.get(k, 0.0), write.get(k, 0.0)
            e["fetch_kib_raw"] = f
            e["write_kib"] = w
            e["hbm_bytes_per_launch"] = int((2 * f + w) * 1024)
        out["kernels"][key] = e
    os.makedirs(os.path.dirname(dst_prefix) or ".", exist_ok=True)
    json.dump(out, open(dst_prefix + "_pmc.json", "w"), indent=1)
    json.dump(out, open(os.path.join(os.path.dirname(dst_prefix), "pmc_latest.json"), "w"), indent=1)
    with open(dst_prefix + "_kernel_stats.csv", "w") as f:
        f.write(open(os.path.join(src, "trace", "run_kernel_stats.csv")).read())
    for k, e in out["kernels"].items():
        print(f"{k:28s} calls {e['calls']:7d} avg {e['avg_ns']/1e3:9.1f} us  "
              f"traffic/launch {e.get('hbm_bytes_per_launch', 0)/1e6:9.2f} MB")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
