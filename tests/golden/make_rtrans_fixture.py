"""Golden rough-transmittance slices for roughplastic, from the reference's precomputed tables.

Reads the reference data files data/microfacet/{beckmann,ggx}.dat (MTS_TRANSMITTANCE format, read
as test data) and restates src/bsdfs/rtrans.h's reductions for a constant (eta, alpha) material, as
RoughPlastic::configure does (roughplastic.cpp:283-299):
  external = RoughTransmittance(type); setEta(eta); setAlpha(alpha)   -> 1D table over warped cos
  internal = clone; setEta(1/eta);  Fdr = 1 - internal.evalDiffuse(alpha)
with Mitsuba's Catmull-Rom evalCubicInterp1D/2D/3D (src/libcore/spline.cpp:23-60,236-304,379-452).
Writes tests/golden/rtrans_slices.npz: per case the 100-entry external table, the external
diffuse transmittance and the internal Fdr.  Run here (needs /root/reference); the output is
committed.
"""
import os
import struct
import sys

import numpy as np

REF = "/root/reference/data/microfacet"
CASES = [  # (distribution, eta, alpha)
    ("beckmann", 1.49 / 1.000277, 0.7),  # test_bsdf.xml:133-136 (polypropylene / air defaults)
    ("beckmann", 1.5, 0.1),
    ("ggx", 1.5, 0.2),
    ("ggx", 1.33, 0.4),
]


def load(name):
    b = open(os.path.join(REF, name + ".dat"), "rb").read()
    assert b[:17] == b"MTS_TRANSMITTANCE"
    ne, na, nt = struct.unpack("<QQQ", b[17:41])
    emin, emax, amin, amax = struct.unpack("<4f", b[41:57])
    raw = np.frombuffer(b[57:], np.float32)
    assert raw.size == 2 * ne * na * (nt + 1)
    raw = raw.reshape(2 * ne, na, nt + 1)
    trans = raw[:, :, :nt].astype(np.float32)   # [2*eta][alpha][theta]
    diff = raw[:, :, nt].astype(np.float32)     # [2*eta][alpha]
    return dict(ne=ne, na=na, nt=nt, emin=emin, emax=emax, amin=amin, amax=amax, trans=trans, diff=diff)


def knot_weights(p, size):
    """spline.cpp:236-282 weights for one dimension (no extrapolation)."""
    if not (0.0 <= p <= 1.0):
        return None, None
    t = np.float32(p) * np.float32(size - 1)
    k = min(int(t), size - 2)
    t = np.float32(t - np.float32(k))
    t2, t3 = t * t, t * t * t
    w = [np.float32(0), 2 * t3 - 3 * t2 + 1, -2 * t3 + 3 * t2, np.float32(0)]
    d0, d1 = t3 - 2 * t2 + t, t3 - t2
    if k > 0:
        w[2] += np.float32(0.5) * d0
        w[0] -= np.float32(0.5) * d0
    else:
        w[2] += d0
        w[1] -= d0
    if k + 2 < size:
        w[3] += np.float32(0.5) * d1
        w[1] -= np.float32(0.5) * d1
    else:
        w[2] += d1
        w[1] -= d1
    return k, [np.float32(x) for x in w]


def cubic_nd(p, data):
    """evalCubicInterp{1,2,3}D: data indexed [z][y][x] with p = (x, y, z)."""
    dims = data.shape[::-1]
    kw = [knot_weights(p[d], dims[d]) for d in range(len(p))]
    if any(k is None for k, _ in kw):
        return np.float32(0)
    res = np.float32(0)
    idx = np.ndindex(*([4] * len(p)))
    for off in sorted(idx, key=lambda o: o[::-1]):
        w = np.float32(1)
        for d in range(len(p)):
            w = w * kw[d][1][off[d]] if d else kw[d][1][off[d]]
        # spline.cpp multiplies innermost weight last: wx * (wy * wz)
        if len(p) == 2:
            w = kw[0][1][off[0]] * kw[1][1][off[1]]
        elif len(p) == 3:
            w = kw[0][1][off[0]] * (kw[1][1][off[1]] * kw[2][1][off[2]])
        if w == 0:
            continue
        pos = tuple(kw[d][0] + off[d] - 1 for d in range(len(p)))[::-1]
        res = np.float32(res + data[pos] * w)
    return res


def cubic1d(x, v):
    """spline.cpp:23-60."""
    n = len(v)
    if not (0.0 <= x <= 1.0):
        return np.float32(0)
    t = np.float32(x) * np.float32(n - 1)
    k = max(0, min(int(t), n - 2))
    f0, f1 = v[k], v[k + 1]
    d0 = np.float32(0.5) * (v[k + 1] - v[k - 1]) if k > 0 else v[k + 1] - v[k]
    d1 = np.float32(0.5) * (v[k + 2] - v[k]) if k + 2 < n else v[k + 1] - v[k]
    t = np.float32(t - np.float32(k))
    t2, t3 = t * t, t * t * t
    return np.float32((2 * t3 - 3 * t2 + 1) * f0 + (-2 * t3 + 3 * t2) * f1 + (t3 - 2 * t2 + t) * d0 + (t3 - t2) * d1)


def warp(v, lo, hi):
    return np.float32(np.power(np.float32((v - lo) / (hi - lo)), np.float32(0.25)))


def slices(T, eta, alpha):
    ne, na, nt = T["ne"], T["na"], T["nt"]

    def set_eta(e):
        block = 0
        if e < 1:
            block, e = 1, 1.0 / e
        e = max(e, T["emin"])
        we = warp(e, T["emin"], T["emax"])
        tr = T["trans"][block * ne:(block + 1) * ne]   # [eta][alpha][theta]
        df = T["diff"][block * ne:(block + 1) * ne]    # [eta][alpha]
        da, dt = np.float32(1.0 / (na - 1)), np.float32(1.0 / (nt - 1))
        new_t = np.zeros((na, nt), np.float32)
        new_d = np.zeros(na, np.float32)
        for i in range(na):
            for j in range(nt):
                new_t[i, j] = cubic_nd((j * dt, i * da, we), tr)
            new_d[i] = cubic_nd((i * da, we), df)
        return new_t, new_d

    wa = warp(alpha, T["amin"], T["amax"])
    ext_t, ext_d = set_eta(eta)
    dt = np.float32(1.0 / (nt - 1))
    table = np.array([cubic_nd((j * dt, wa), ext_t) for j in range(nt)], np.float32)  # setAlpha
    ext_diff = cubic1d(wa, ext_d)
    int_t, int_d = set_eta(1.0 / eta)
    int_diff = np.clip(cubic1d(wa, int_d), 0, 1)
    return table, np.float32(ext_diff), np.float32(1 - int_diff)


def main():
    out = {}
    tabs = {n: load(n) for n in ("beckmann", "ggx")}
    for i, (dist, eta, alpha) in enumerate(CASES):
        table, ext_diff, fdr = slices(tabs[dist], eta, alpha)
        out[f"case{i}_params"] = np.array([0 if dist == "beckmann" else 1, eta, alpha], np.float64)
        out[f"case{i}_table"] = table
        out[f"case{i}_ext_diffuse"] = np.array([ext_diff])
        out[f"case{i}_fdr_int"] = np.array([fdr])
        print(dist, eta, alpha, "T(cos=1)", table[-1], "T(cos=0.5^4)", table[50], "Fdr_int", fdr, flush=True)
    np.savez(os.path.join(os.path.dirname(os.path.abspath(__file__)), "rtrans_slices.npz"), **out)


if __name__ == "__main__":
    sys.exit(main())
