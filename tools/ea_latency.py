"""Mean memory-side (L2 -> fabric) read latency of the path kernels from a rocprofv3 --pmc pass with
TCC_EA0_RDREQ_sum and TCC_EA0_RDREQ_LEVEL_sum (Little's law: LEVEL / RDREQ cycles), for the bench's
calibration launches (the last N dispatches of each kernel, N from the trace summary or 12).

usage: python tools/ea_latency.py PMC_DIR [N]
"""
import csv
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import base_name  # noqa: E402


def main(d, n=12):
    per = defaultdict(lambda: defaultdict(dict))
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        per[base_name(r["Kernel_Name"])][int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    for k, disp in sorted(per.items()):
        ids = sorted(disp)[-n:]
        req = sum(disp[i].get("TCC_EA0_RDREQ_sum", 0) for i in ids)
        lev = sum(disp[i].get("TCC_EA0_RDREQ_LEVEL_sum", 0) for i in ids)
        if req > 1e5:
            print(f"{k:16s} last {len(ids):3d} dispatches: EA read requests {req / len(ids):14.0f} per launch, "
                  f"mean latency {lev / req:7.1f} cycles")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12)
