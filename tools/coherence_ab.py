"""Ray-order A/B for k_trace: does binning secondary rays by direction octant (or by origin) make
closest-hit traversal faster?  Builds C3 bounce rays on the GPU (pinhole camera rays in 8x8-tile
slot order, then cosine bounces off the geometric normal), and traces each ray set in several
orders with pg_trace_rays.  Run under rocprofv3 --kernel-trace; the launches appear in this order:
  for bounce in (2, 3): for order in ORDERS: REPS launches
  python tools/coherence_ab.py [spp]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pgload  # noqa: E402

pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import Device  # noqa: E402

ORDERS = ["slot", "octant", "octant_morton", "morton", "random"]
REPS = 4


def camera_rays(sc, spp, rng):
    c = sc.camera
    o = np.array(c.origin[:], np.float64)
    f = np.array(c.target[:], np.float64) - o
    f /= np.linalg.norm(f)
    r = np.cross(f, np.array(c.up[:], np.float64))
    r /= np.linalg.norm(r)
    u = np.cross(r, f)
    W, H = c.width, c.height
    tx = np.tan(np.radians(c.fov_x_deg) * 0.5)
    ty = tx * H / W
    # 8x8 pixel tiles, spp samples of a pixel adjacent (the camera queue's slot order)
    ty_, tx_ = np.meshgrid(np.arange(H // 8), np.arange(W // 8), indexing="ij")
    iy, ix = np.meshgrid(np.arange(8), np.arange(8), indexing="ij")
    px = (tx_.reshape(-1, 1) * 8 + ix.reshape(1, -1)).reshape(-1)
    py = (ty_.reshape(-1, 1) * 8 + iy.reshape(1, -1)).reshape(-1)
    px = np.repeat(px, spp) + rng.random(len(px) * spp)
    py = np.repeat(py, spp) + rng.random(len(py) * spp)
    sx = (2 * px / W - 1) * tx
    sy = (1 - 2 * py / H) * ty
    d = f[None] + sx[:, None] * r[None] + sy[:, None] * u[None]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.zeros((len(d), 8), np.float32)
    rays[:, 0:3] = o
    rays[:, 3] = 1e-4
    rays[:, 4:7] = d
    rays[:, 7] = np.inf
    return rays


def bounce(sc, rays, hits, rng):
    tri = hits[:, 1].view(np.uint32)
    m = tri != 0xFFFFFFFF
    rays, hits, tri = rays[m], hits[m], tri[m]
    P = sc.positions[sc.indices[tri]]  # (n, 3, 3)
    n = np.cross(P[:, 1] - P[:, 0], P[:, 2] - P[:, 0])
    n /= np.maximum(np.linalg.norm(n, axis=1, keepdims=True), 1e-30)
    n *= -np.sign(np.sum(n * rays[:, 4:7], 1, keepdims=True))
    x = rays[:, 0:3] + hits[:, 0:1] * rays[:, 4:7]
    # cosine-weighted about n
    u1, u2 = rng.random(len(n)), rng.random(len(n))
    rr, ph = np.sqrt(u1), 2 * np.pi * u2
    a = np.where(np.abs(n[:, 0:1]) > 0.9, [[0, 1, 0]], [[1, 0, 0]])
    t = np.cross(n, a)
    t /= np.linalg.norm(t, axis=1, keepdims=True)
    b = np.cross(n, t)
    d = (rr * np.cos(ph))[:, None] * t + (rr * np.sin(ph))[:, None] * b + np.sqrt(1 - u1)[:, None] * n
    out = np.zeros((len(d), 8), np.float32)
    out[:, 0:3] = x + 1e-4 * n
    out[:, 3] = 1e-4
    out[:, 4:7] = d
    out[:, 7] = np.inf
    return out


def morton(x, lo, hi):
    q = np.clip(((x - lo) / (hi - lo) * 1023).astype(np.int64), 0, 1023)
    code = np.zeros(len(x), np.int64)
    for bit in range(10):
        for k in range(3):
            code |= ((q[:, k] >> bit) & 1) << (3 * bit + k)
    return code


def ordered(rays, order, lo, hi, rng):
    octant = ((rays[:, 4] < 0).astype(np.int64) | (rays[:, 5] < 0) << 1 | (rays[:, 6] < 0) << 2)
    if order == "slot":
        return rays
    if order == "octant":
        return rays[np.argsort(octant, kind="stable")]
    if order == "octant_morton":
        return rays[np.argsort((octant << 30) | morton(rays[:, 0:3], lo, hi), kind="stable")]
    if order == "morton":
        return rays[np.argsort(morton(rays[:, 0:3], lo, hi), kind="stable")]
    return rays[rng.permutation(len(rays))]


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    rng = np.random.default_rng(7)
    sc = pg.scenes.ajar_door(1280, 720)
    d = Device(pg.capi.default_config())
    d.upload(sc)
    lo, hi = (np.asarray(v, np.float64) for v in sc.bounds())
    r = camera_rays(sc, spp, rng)
    h = d.trace_rays(r)
    for b in (2, 3):
        r = bounce(sc, r, h, rng)
        sets = {o: ordered(r, o, lo, hi, rng) for o in ORDERS}
        for o in ORDERS:
            for _ in range(REPS):
                hh = d.trace_rays(sets[o])
            print(f"bounce {b} {o}: {len(r)} rays, hit frac {(hh[:, 1].view(np.uint32) != 0xFFFFFFFF).mean():.4f}",
                  flush=True)
        h = d.trace_rays(r)


if __name__ == "__main__":
    main()
