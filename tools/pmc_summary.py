"""Summarise a tools/profile.sh output directory into profiles/.

Per kernel: calls, average duration (kernel trace), and HBM traffic per launch from the separate
FETCH_SIZE / WRITE_SIZE passes.  gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts
64-B units for 128-B requests, i.e. half the bytes of wide (16 B/lane) reads -> doubled here;
WRITE_SIZE is taken as-is.  Both counters are in KiB.

bench.py measures the kernel roofline on a one-lane context after the timed region (the timed job
overlaps three lanes, so per-launch durations there include other lanes' work).  That context's
stream is the last one to launch k_trace, so the path kernels (k_trace, k_shade_all, k_rays; the
unfused k_shade, k_shadow when fusion is off) are summarised over that stream only ("calibration"
view) as well as over the whole run.
usage: python tools/pmc_summary.py gpurun_out/prof_rNN profiles/rNN
"""
import csv
import json
import os
import subprocess
import sys
from collections import defaultdict

PATH_KERNELS = ("k_trace", "k_shade", "k_shadow", "k_shade_all", "k_rays", "k_vflight", "k_vvertex", "k_vnee")


def base_name(n):
    return n.split("(")[0].split("<")[0].replace("void ", "").strip()


def rows_of(path):
    return list(csv.DictReader(open(path))) if os.path.exists(path) else []


def calibration_stream(rows):
    """the stream of the last k_trace launch (surface path) or, for the volumetric wavefront, of the last
    k_vflight launch: bench.py's calibration context runs after the timed region"""
    tr = [r for r in rows if base_name(r["Kernel_Name"]) == "k_trace" and "Stream_Id" in r]
    if not tr:
        tr = [r for r in rows if base_name(r["Kernel_Name"]) == "k_vflight" and "Stream_Id" in r]
    if not tr:
        return None
    return max(tr, key=lambda r: int(r.get("Start_Timestamp", r.get("Dispatch_Id", 0))))["Stream_Id"]


def load_counter(path, name):
    """per-kernel counter values in dispatch order"""
    acc = defaultdict(list)
    for row in rows_of(path):
        if row["Counter_Name"] == name:
            acc[base_name(row["Kernel_Name"])].append((int(row["Dispatch_Id"]), float(row["Counter_Value"])))
    return {k: [v for _, v in sorted(l)] for k, l in acc.items()}


def revision():
    """git HEAD of the tree that was uploaded for the profile (run this right after the profile call);
    PG_REVISION names it when the summary runs on the GPU box (no .git there)."""
    if os.environ.get("PG_REVISION"):
        return os.environ["PG_REVISION"]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    try:
        head = subprocess.run(["git", "-C", root, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                              text=True, timeout=10).stdout.strip()
        dirty = subprocess.run(["git", "-C", root, "status", "--porcelain", "--untracked-files=no", "--", "*.hip",
                                "*.cpp", "*.h", "*.py"], capture_output=True, text=True, timeout=10).stdout.strip()
        return head + ("+dirty" if dirty else "") if head else None
    except (OSError, subprocess.SubprocessError):
        return None


def mean(v):
    return sum(v) / len(v) if v else 0.0


def main(src, dst_prefix):
    trace = rows_of(os.path.join(src, "trace", "run_kernel_trace.csv"))
    cal = calibration_stream(trace)
    stats = defaultdict(lambda: {"calls": 0, "total_ns": 0.0})
    cstats = defaultdict(lambda: {"calls": 0, "total_ns": 0.0})
    for r in trace:
        k = base_name(r["Kernel_Name"])
        dt = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        stats[k]["calls"] += 1
        stats[k]["total_ns"] += dt
        if r.get("Stream_Id") == cal:
            cstats[k]["calls"] += 1
            cstats[k]["total_ns"] += dt
    # the counter CSVs carry no stream id; the calibration pass is the last (deterministic) work of
    # the run, so its launches are the last `calibration_calls` dispatches of each path kernel
    fetch = load_counter(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = load_counter(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    out = {"source": src, "revision": revision(), "correction": "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per launch",
           "calibration_stream": cal, "kernels": {}}
    for k, s in sorted(stats.items(), key=lambda kv: -kv[1]["total_ns"]):
        e = {"calls": s["calls"], "avg_ns": s["total_ns"] / s["calls"], "total_ns": s["total_ns"]}
        if k in fetch or k in write:
            f, w = mean(fetch.get(k, [])), mean(write.get(k, []))
            e["fetch_kib_raw"], e["write_kib"] = f, w
            e["hbm_bytes_per_launch_all"] = int((2 * f + w) * 1024)
        if k in PATH_KERNELS and cstats[k]["calls"]:
            n = cstats[k]["calls"]
            e["calibration_calls"] = n
            e["calibration_avg_ns"] = cstats[k]["total_ns"] / n
            if k in fetch or k in write:
                f, w = mean(fetch.get(k, [])[-n:]), mean(write.get(k, [])[-n:])
                e["calibration_fetch_kib_raw"], e["calibration_write_kib"] = f, w
                e["hbm_bytes_per_launch"] = int((2 * f + w) * 1024)
        elif "hbm_bytes_per_launch_all" in e:
            e["hbm_bytes_per_launch"] = e["hbm_bytes_per_launch_all"]
        out["kernels"][k] = e
    os.makedirs(os.path.dirname(dst_prefix) or ".", exist_ok=True)
    json.dump(out, open(dst_prefix + "_pmc.json", "w"), indent=1)
    vol = "k_volpath" in out["kernels"] or "k_vflight" in out["kernels"]
    latest = "pmc_volpath_latest.json" if vol else "pmc_latest.json"  # read by bench.py
    json.dump(out, open(os.path.join(os.path.dirname(dst_prefix), latest), "w"), indent=1)
    with open(dst_prefix + "_kernel_stats.csv", "w") as f:
        f.write(open(os.path.join(src, "trace", "run_kernel_stats.csv")).read())
    for k, e in out["kernels"].items():
        cal_s = (f"  calibration: {e['calibration_calls']} calls avg {e['calibration_avg_ns']/1e3:8.1f} us"
                 if "calibration_avg_ns" in e else "")
        print(f"{k:28s} calls {e['calls']:7d} avg {e['avg_ns']/1e3:9.1f} us  "
              f"traffic/launch {e.get('hbm_bytes_per_launch', 0)/1e6:9.2f} MB{cal_s}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
