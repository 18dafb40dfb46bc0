"""Depth statistics of a serialized SD-tree (pg_sdtree.cpp SdTree::serialize): per D-tree the leaf-quadrant
depth a query reaches, weighted by energy (where guided samples land) and by area (a direction drawn
uniformly, e.g. a BSDF sample's pdf query), every D-tree weighted alike.

  python tools/dtree_depths.py TREE.npy
"""
import sys

import numpy as np


def main(path):
    b = np.load(path).tobytes()
    u32 = lambda o, n: np.frombuffer(b, np.uint32, n, o)
    off = 16 + 32
    ns, nl, nq, nb = u32(off, 4)
    off += 16 + 8 * int(ns)
    meta = u32(off, 8 * int(nl)).reshape(-1, 8)
    off += 32 * int(nl)
    q = np.frombuffer(b, np.uint32, 8 * int(nq), off).reshape(-1, 8)
    qsum = q[:, :4].view(np.float32)
    qch = q[:, 4:]
    we, wa, wsum = np.zeros(40), np.zeros(40), 0.0
    for i in range(int(nl)):
        base, cnt = int(meta[i, 0]), int(meta[i, 2])
        count = 1.0  # every D-tree alike (the record counts are cleared by the refit)
        total = float(qsum[base].sum())
        stack = [(base, 0, 1.0)]
        while stack:
            n, d, area = stack.pop()
            s = qsum[n]
            tot = float(s.sum())
            for k in range(4):
                c = int(qch[n, k])
                if c:
                    stack.append((c, d + 1, area / 4))
                else:
                    we[d + 1] += count * (float(s[k]) / total if total > 0 else 0.0)
                    wa[d + 1] += count * area / 4
        wsum += count
    we /= wsum
    wa /= wsum
    dd = np.arange(40)
    print(f"S-tree nodes {int(ns)}, D-trees {int(nl)}, sampling D-tree nodes {int(nq)}")
    print(f"energy-weighted leaf depth: mean {float((we * dd).sum()):.2f}; P(depth >= k) for k = 1..12:",
          " ".join(f"{float(we[k:].sum()):.2f}" for k in range(1, 13)))
    print(f"area-weighted leaf depth:   mean {float((wa * dd).sum()):.2f}; P(depth >= k) for k = 1..12:",
          " ".join(f"{float(wa[k:].sum()):.2f}" for k in range(1, 13)))


if __name__ == "__main__":
    main(sys.argv[1])
