"""Run-to-run determinism of the guided C3 training (two fresh contexts in one process): per
iteration, md5 of the sorted record set, the film and the refit SD-tree.
  python tools/det_check.py [--runs 2] [--width 1280 --height 720]"""
import argparse
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pgload  # noqa: E402


def md5(a):
    return hashlib.md5(np.ascontiguousarray(a).tobytes()).hexdigest()[:10]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--train", type=int, default=5)
    a = ap.parse_args()
    pg = pgload.load()
    from mitsuba_path_guiding_amd.integrator import Device
    sc = pg.scenes.ajar_door(a.width, a.height)
    runs = []
    for r in range(a.runs):
        d = Device(pg.capi.default_config(guiding=1))
        d.upload(sc)
        off, rows = 0, []
        for it in range(a.train):
            d.render_pass(2 ** it, off, record=True)
            off += 2 ** it
            rec = d.get_records().reshape(-1, 32)
            srt = rec[np.lexsort(rec.T[::-1])]
            film = d.read_film()[0]
            d.splat_local()
            d.refit(it)
            tree = d.get_sdtree()
            rows.append((len(rec), md5(srt), md5(film), md5(tree)))
            print(f"run {r} it {it}: records {len(rec)} rec {rows[-1][1]} film {rows[-1][2]} tree {rows[-1][3]}",
                  flush=True)
            d.reset_film()
        d.close()
        runs.append(rows)
    same = all(x == runs[0] for x in runs)
    print("deterministic" if same else "NONDETERMINISTIC")


if __name__ == "__main__":
    main()
