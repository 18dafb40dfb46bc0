"""Summarise tools/coherence_ab.py's k_trace_rays launches from a rocprofv3 kernel trace CSV.
  python tools/coherence_summary.py TRACE.csv"""
import csv
import sys

ORDERS = ["slot", "octant", "octant_morton", "morton", "random"]
REPS = 4
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_trace_rays" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
# launch 0: camera rays; then per bounce: ORDERS x REPS, one unordered re-trace
k = 1
for b in (2, 3):
    for o in ORDERS:
        ds = dur[k:k + REPS]
        k += REPS
        print(f"bounce {b} {o:14s} us/launch min {min(ds):9.1f} med {sorted(ds)[len(ds) // 2]:9.1f}")
    k += 1
