"""Analytic images for the reference's two-disk test scenes (fixture generator; test data only).

data/tests/test_bidir_0.xml: two coaxial unit disks 2 apart.  The receiver at z = -1 faces +z
(diffuse, the default reflectance 0.5); the emitter at z = +1 is flipped to face -z (diffuse 0.5,
area emitter of radiance 1).  test_bidir_2.xml adds a homogeneous medium (sigma_a = 1, sigma_s = 0)
entered through an index-matched disk at z = 0 and left at the emitter, so every receiver-emitter
segment spends half its length in the medium: transmittance exp(-|y - x| / 2).

A pinhole camera at z = -0.4 looks straight down at the receiver (90 deg, 32 x 32 pixels): every
pixel sees the receiver at radius <= 0.85, with radiance rho / pi * E(r).  E = direct + reflected:

  direct     the loader's 256-gon emitter, exactly: Lambert's polygon formula in vacuum
             (E = 1/2 sum_k Theta_k n.Gamma_k), a fan-triangle Gauss-Legendre rule (Duffy map,
             12 x 12 nodes per triangle) through the medium;
  reflected  the interreflection series between the two rho = 0.5 disks (Neumann series of the
             radial integral equation on Gauss-Legendre nodes, ring kernel in closed form in vacuum,
             2 x 64-node angular quadrature through the medium); ~3 % of the direct term, so the
             disk-for-polygon approximation there is below 1e-5 relative.

The per-pixel expectation averages rho / pi * E over 16 x 16 sub-pixel positions (E is smooth).
bidir2_refmis_image is the expectation of the reference's volpath estimator with NEE on, whose MIS
weights do not sum to one behind an index-matched surface (direct_medium, mis="reference").
All float64.  Writes tests/golden/bidir_analytic.npz.
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
N_SEG = 256          # mitsuba_xml: disk = 4 * sphere_res[0] segments (default 64)
H = 2.0              # receiver z = -1, emitter z = +1
RHO = 0.5            # diffuse default reflectance
SIGMA = 1.0          # test_bidir_2 sigma_a
CAM = dict(origin=(0.0, 0.0, -0.4), target=(0.0, 0.0, -1.0), up=(0.0, 1.0, 0.0), fov_x=90.0, width=32, height=32)


def polygon():
    a = np.arange(N_SEG) * 2 * np.pi / N_SEG
    return np.stack([np.cos(a), np.sin(a)], 1)


def direct_vacuum(r):
    """Irradiance at (r, 0, -1) (normal +z) from the radiance-1 polygon at z = +1 (Lambert)."""
    P = polygon()
    out = np.zeros(len(r))
    for i, x in enumerate(r):
        v = np.concatenate([P - [x, 0.0], np.full((N_SEG, 1), H)], 1)
        u = v / np.linalg.norm(v, axis=1, keepdims=True)
        w = np.roll(u, -1, 0)
        theta = np.arccos(np.clip((u * w).sum(1), -1, 1))
        c = np.cross(u, w)
        gam = c[:, 2] / np.linalg.norm(c, axis=1)
        out[i] = abs(0.5 * (theta * gam).sum())
    return out


def direct_medium(r, sigma=SIGMA, m=12, mis=None):
    """Same through the medium: fan triangles (centre, p_k, p_k+1), Duffy map, m x m Gauss-Legendre.

    mis="reference": the expectation of the reference's estimator with next-event estimation on
    (progressive_volpath.cpp: NEE weighted miWeight(dRec.pdf, bsdfPdf), a BSDF-sampled emitter hit
    weighted miWeight(bsdfPdf, pdfEmitterDirect(dRec))).  rayIntersectAndLookForEmitter hands
    dRec.dist = its->t of the LAST segment (records.inl:170-178 setQuery, after ray.o moved to the
    index-matched disk at z = 0), i.e. d / 2 here, so the BSDF side's emitter pdf is 4x too small and
    the two weights sum to more than 1: w_nee(p_n, p_b) + w_bsdf(p_b, p_n / 4) with p_n = d^2 / (A cos)
    the area sampler's solid-angle pdf and p_b = cos / pi the diffuse receiver's."""
    P = polygon()
    area = 0.5 * N_SEG * np.sin(2 * np.pi / N_SEG)
    g, gw = np.polynomial.legendre.leggauss(m)
    g, gw = 0.5 * (g + 1), 0.5 * gw
    U, V = np.meshgrid(g, g, indexing="ij")
    Wt = np.outer(gw, gw)
    a, b = P, np.roll(P, -1, 0)
    # y = u * a + u * v * (b - a), dA = u * |a x (b - a)| du dv
    Y = U[None] [..., None] * a[:, None, None, :] + (U * V)[None][..., None] * (b - a)[:, None, None, :]
    jac = np.abs(a[:, 0] * (b - a)[:, 1] - a[:, 1] * (b - a)[:, 0])[:, None, None] * U[None]
    wts = (Wt[None] * jac).reshape(-1)
    Y = Y.reshape(-1, 2)
    out = np.zeros(len(r))
    for i, x in enumerate(r):
        d2 = (Y[:, 0] - x) ** 2 + Y[:, 1] ** 2 + H * H
        d = np.sqrt(d2)
        f = wts * H * H / (d2 * d2) * np.exp(-sigma * d / 2)
        if mis == "reference":
            cos = H / d
            pn, pb = d2 / (area * cos), cos / np.pi
            pn_last = (d / 2) ** 2 / (area * cos)
            f = f * (pn ** 2 / (pn ** 2 + pb ** 2) + pb ** 2 / (pb ** 2 + pn_last ** 2))
        out[i] = f.sum()
    return out


def ring_kernel(r, s, sigma):
    """k(r, s) = int_0^{2 pi} h^2 / d^4 exp(-sigma d / 2) dphi between radius r of one disk and s of
    the other; closed form for sigma = 0."""
    r, s = np.asarray(r, np.float64)[:, None], np.asarray(s, np.float64)[None, :]
    A = H * H + r * r + s * s
    if sigma == 0:
        B = 2 * r * s
        return 2 * np.pi * H * H * A / (A * A - B * B) ** 1.5
    t, tw = np.polynomial.legendre.leggauss(64)
    phi, pw = 0.5 * np.pi * (t + 1), 0.5 * np.pi * tw
    d2 = A[..., None] - 2 * r[..., None] * s[..., None] * np.cos(phi)
    d = np.sqrt(d2)
    return 2 * (pw * H * H / (d2 * d2) * np.exp(-sigma * d / 2)).sum(-1)


def reflected(r_eval, sigma, n=96, source=None):
    """Interreflected part of the receiver irradiance (disk model): E_r = E_d + K rho/pi E_e,
    E_e = K rho/pi E_r, iterated to convergence; returns E_r - E_d at r_eval.  source(r): the direct
    term the receiver's own vertices estimate (default: the disk's irradiance)."""
    x, w = np.polynomial.legendre.leggauss(n)
    x, w = 0.5 * (x + 1), 0.5 * w
    K = ring_kernel(x, x, sigma) * (x * w)[None, :]  # (K f)(r_i) = sum_j f(s_j) k(r_i, s_j) s_j w_j
    Ed = K @ np.ones(n) if source is None else source(x)  # direct irradiance of the radiance-1 emitter
    Er = Ed.copy()
    for _ in range(200):
        Ee = K @ (RHO / np.pi * Er)
        new = Ed + K @ (RHO / np.pi * Ee)
        if np.max(np.abs(new - Er)) < 1e-15:
            break
        Er = new
    Ee = K @ (RHO / np.pi * Er)
    Ke = ring_kernel(r_eval, x, sigma) * (x * w)[None, :]
    return Ke @ (RHO / np.pi * Ee)


def pixel_radii(sub=16):
    """Receiver radius seen through each sub-pixel position of the camera (k_camera's mapping)."""
    W, Hh = CAM["width"], CAM["height"]
    tan = np.tan(np.radians(CAM["fov_x"]) / 2)
    aspect = W / Hh
    dist = CAM["origin"][2] - CAM["target"][2]
    j = (np.arange(sub) + 0.5) / sub
    px = (np.arange(W)[:, None] + j[None, :]).reshape(-1)
    py = (np.arange(Hh)[:, None] + j[None, :]).reshape(-1)
    sx, sy = px / W, py / Hh
    X = (1 - 2 * sx) * tan
    Y = (1 - 2 * sy) / aspect * tan
    R = dist * np.sqrt(X[None, :] ** 2 + Y[:, None] ** 2)  # (H*sub, W*sub)
    return R


def main():
    rr = np.linspace(0.0, 0.9, 181)
    out = {"radius": rr, "n_segments": N_SEG, "rho": RHO, "sigma_a": SIGMA,
           "camera": np.array([*CAM["origin"], *CAM["target"], *CAM["up"], CAM["fov_x"], CAM["width"], CAM["height"]])}
    R = pixel_radii()
    assert R.max() < 0.9
    ref_mis = lambda r: direct_medium(r, mis="reference")  # noqa: E731
    for name, sigma, direct, src in (("bidir0", 0.0, direct_vacuum, None), ("bidir2", SIGMA, direct_medium, None),
                                     ("bidir2_refmis", SIGMA, ref_mis, ref_mis)):
        Ed = direct(rr)
        Ei = reflected(rr, sigma, source=src)
        E = Ed + Ei
        L = RHO / np.pi * np.interp(R, rr, E)
        img = L.reshape(CAM["height"], 16, CAM["width"], 16).mean((1, 3))
        out[f"{name}_direct"], out[f"{name}_reflected"], out[f"{name}_image"] = Ed, Ei, img
        print(f"{name}: E(0) = {E[0]:.8f} (direct {Ed[0]:.8f}, reflected {Ei[0]:.3e}); image mean {img.mean():.8f}")
    # checks of the quadratures: the polygon direct term against the disk's closed form at r = 0
    # (pi / (1 + h^2) for the disk; the 256-gon has 1e-4 less area), vacuum vs sigma -> 0
    print("disk closed form at r=0:", np.pi / (1 + H * H), " polygon:", out["bidir0_direct"][0])
    assert abs(direct_medium(np.array([0.3]), sigma=0.0)[0] - direct_vacuum(np.array([0.3]))[0]) < 1e-9
    np.savez_compressed(os.path.join(HERE, "bidir_analytic.npz"), **out)


if __name__ == "__main__":
    main()
