"""Summarise the FETCH_SIZE calibration (tools/fetch_calib.hip) run under rocprofv3 counter passes.

usage: python tools/fetch_calib_summary.py RUN_DIR OUT.json
RUN_DIR holds `cases.jsonl` (the program's stdout: true bytes, 128-B lines and HIP-event time per case) and
one rocprofv3 --pmc output directory per pass (`fetch/`, `req/`, `hit/`), each with run_counter_collection.csv.
Every case launches its kernel twice (warm, timed); the second dispatch is used.  Per case it reports
FETCH_SIZE bytes (the counter's KiB x 1024, raw: no correction) per true byte and per touched 128-B line,
TCC_EA0_RDREQ per line, and the L2 hit rate, so the path kernels' FETCH_SIZE can be converted with the
factor of their own access width instead of the blanket x2 of MI355X_MICROARCH.md §HBM.
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict


def case_of(kernel_name):
    """the CASE template argument (the first one) of a k_cal_* kernel, or None"""
    m = re.search(r"k_cal_(stream|gather|reuse|scatter16)<(\d+)", kernel_name)
    return int(m.group(2)) if m else None


def counters(path):
    """{case id: {counter: value of the second dispatch}}"""
    per = defaultdict(lambda: defaultdict(dict))  # case -> dispatch -> counter -> value
    if not os.path.exists(path):
        return {}
    for r in csv.DictReader(open(path)):
        c = case_of(r["Kernel_Name"])
        if c is None:
            continue
        per[c][int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    out = {}
    for c, d in per.items():
        ids = sorted(d)
        out[c] = d[ids[-1]]  # the timed (second) launch
    return out


# the CASE ids of fetch_calib.hip in launch order
CASE_IDS = [0, 1, 10, 11, 12, 13, 14, 15, 20, 21, 22, 23]


def main(run, dst):
    cases = [json.loads(l) for l in open(os.path.join(run, "cases.jsonl")) if l.startswith("{\"case\"")]
    cnt = {}
    for p in sorted(os.listdir(run)):
        f = os.path.join(run, p, "run_counter_collection.csv")
        for c, v in counters(f).items():
            cnt.setdefault(c, {}).update(v)
    rows = []
    for cid, cs in zip(CASE_IDS, cases):
        v = cnt.get(cid, {})
        e = dict(cs)
        e["counters"] = v
        if "FETCH_SIZE" in v:
            fb = v["FETCH_SIZE"] * 1024
            e["fetch_bytes_raw"] = fb
            e["fetch_per_true_byte"] = round(fb / cs["true_bytes"], 4)
            e["fetch_per_line"] = round(fb / max(cs["lines_128"], 1), 2)
        if "TCC_EA0_RDREQ_sum" in v:
            e["ea_rdreq_per_line"] = round(v["TCC_EA0_RDREQ_sum"] / max(cs["lines_128"], 1), 3)
        if "TCC_EA0_RDREQ_LEVEL_sum" in v and v.get("TCC_EA0_RDREQ_sum"):
            # Little's law over the L2's memory-side read queue: mean cycles a read request is outstanding
            e["ea_read_latency_cycles"] = round(v["TCC_EA0_RDREQ_LEVEL_sum"] / v["TCC_EA0_RDREQ_sum"], 1)
        if "TCC_HIT_sum" in v and "TCC_MISS_sum" in v:
            e["l2_hit"] = round(v["TCC_HIT_sum"] / max(v["TCC_HIT_sum"] + v["TCC_MISS_sum"], 1), 4)
        rows.append(e)
        print(f"{cs['case']:28s} true {cs['true_bytes']/1e6:9.1f} MB  {cs['gbs']:8.1f} GB/s  "
              f"fetch/true {e.get('fetch_per_true_byte', float('nan')):6.3f}  fetch/line {e.get('fetch_per_line', float('nan')):7.1f} B  "
              f"EA req/line {e.get('ea_rdreq_per_line', float('nan')):6.3f}  L2 hit {e.get('l2_hit', float('nan')):.3f}  "
              f"EA lat {e.get('ea_read_latency_cycles', float('nan')):7.1f}")
    json.dump({"source": run, "cases": rows}, open(dst, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
