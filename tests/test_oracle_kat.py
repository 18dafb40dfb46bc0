"""Pins the CPU oracle against the reference's own known-answer tests and fixtures.

  * src/tests/test_dgeom.cpp:36-121 — triangle-hit differential geometry (tests/golden/dgeom_kat.json)
  * src/tests/test_kd.cpp:86-130 + data/tests/bunny.ply — rays between random points of the bunny's
    bounding sphere; the oracle's BVH must find the same closest hits as a brute-force TriAccel-free
    (Moeller-Trumbore, float64) reference over all 69,451 faces.
  * determinism of the oracle film against its committed golden output.
"""
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _single_triangle_scene(pg, V, N):
    s = pg.scenes.Scene()
    m = s.add_material(pg.scenes.material("diffuse"))
    s.add_mesh(np.asarray(V, np.float32), np.array([[0, 1, 2]], np.uint32), N, material=m)
    s.set_camera((0.2, 0.2, -2), (0.2, 0.2, 0), (0, 1, 0), 40, 8, 8)
    return s.finalize()


def dgeom_scene(pg, case):
    V = np.array(case["vertices"], np.float32)
    if case["normals"] is None:
        N = np.tile(np.array([[0, 0, 1]], np.float32), (3, 1))  # TriMesh face normal
    else:
        N = np.array(case["normals"], np.float32)
    return _single_triangle_scene(pg, V, N)


def check_dgeom_case(case, rec, bary):
    """One KAT case against a hit record (n x 16 layout of pg_hit_records / oracle_hit_records: p, t, geoN,
    shN, shading frame s, wi) and the hit's barycentrics (b1, b2)."""
    eps = case["eps"]
    p, geoN, shN, shS, wi = rec[0:3], rec[4:7], rec[7:10], rec[10:13], rec[13:16]
    assert np.allclose(p, case["p"], atol=eps), (case["name"], p)
    assert np.allclose(geoN, case["geoN"], atol=eps), (case["name"], geoN)
    b = np.array([1 - bary[0] - bary[1], bary[0], bary[1]], np.float64)
    if "bary" in case:
        assert np.allclose(b, case["bary"], atol=eps), (case["name"], b)
    # its.uv: interpolated texcoords, or (b1, b2) without them (skdtree.h:398-405)
    T = case["texcoords"]
    uv = b[1:] if T is None else (np.array(T, np.float64) * b[:, None]).sum(0)
    assert np.allclose(uv, case["uv"], atol=eps), (case["name"], uv)
    if "shN_weights" in case:  # normalize(n0*.7 + n1*.1 + n2*.2)
        n = (np.array(case["normals"], np.float64) * np.array(case["shN_weights"])[:, None]).sum(0)
        n /= np.linalg.norm(n)
    else:
        n = np.array(case["shN"], np.float64)
    assert np.allclose(shN, n, atol=eps), (case["name"], shN, n)
    # shading tangent: computeShadingFrame(n, dpdu) = normalize(dpdu - n dot(n, dpdu)) (:106-107,160-161)
    if "dpdu" in case:
        dpdu = np.array(case["dpdu"], np.float64)
        s = dpdu - n * n.dot(dpdu)
        s /= np.linalg.norm(s)
        assert np.allclose(shS, s, atol=eps), (case["name"], shS, s)
        t = np.cross(n, s)
        d = -np.array(case["ray_d"], np.float64)
        assert np.allclose(wi, [d.dot(s), d.dot(t), d.dot(n)], atol=eps), (case["name"], wi)


def test_dgeom_kat(pg, O):
    kat = json.load(open(os.path.join(GOLDEN, "dgeom_kat.json")))
    assert [c["kat"] for c in kat["cases"]] == ["test_dgeom.cpp:35-67", "test_dgeom.cpp:69-120",
                                                "test_dgeom.cpp:122-177"]
    for case in kat["cases"]:
        osc = O.OracleScene(pg.capi, dgeom_scene(pg, case))
        r = np.array([[*case["ray_o"], 1e-4, *case["ray_d"], np.inf]], np.float32)
        h = osc.intersect(r)[0]
        assert h[15].view(np.uint32) == 0
        assert np.allclose(h[10:13], case.get("dpdu", [1, 0, 0]), atol=case["eps"])  # side1 = p1 - p0
        check_dgeom_case(case, osc.hit_records(r)[0], h[13:15])


def _brute_force(V, F, o, d):
    """float64 Moeller-Trumbore over all faces; returns (t, face) per ray."""
    p0, p1, p2 = V[F[:, 0]].astype(np.float64), V[F[:, 1]].astype(np.float64), V[F[:, 2]].astype(np.float64)
    e1, e2 = p1 - p0, p2 - p0
    ts = np.full(len(o), np.inf)
    fs = np.full(len(o), -1)
    for i in range(len(o)):
        pv = np.cross(d[i], e2)
        det = np.einsum("ij,ij->i", e1, pv)
        ok = np.abs(det) > 1e-12
        inv = np.where(ok, 1.0 / np.where(ok, det, 1.0), 0.0)
        tv = o[i] - p0
        u = np.einsum("ij,ij->i", tv, pv) * inv
        qv = np.cross(tv, e1)
        v = (qv @ d[i]) * inv
        t = np.einsum("ij,ij->i", e2, qv) * inv
        hit = ok & (u >= 0) & (v >= 0) & (u + v <= 1) & (t > 1e-6)
        if hit.any():
            j = np.argmin(np.where(hit, t, np.inf))
            ts[i], fs[i] = t[j], j
    return ts, fs


def _bunny_scene(pg):
    z = np.load(os.path.join(GOLDEN, "bunny.npz"))
    V, F = z["positions"], z["faces"]
    s = pg.scenes.Scene()
    m = s.add_material(pg.scenes.material("diffuse"))
    s.add_mesh(V, F, material=m)
    c = V.mean(0)
    s.set_camera(tuple(c + np.array([0, 0, 1.0])), tuple(c), (0, 1, 0), 40, 8, 8)
    return s.finalize(), V, F


def bunny_sphere_rays(V, n, seed):
    """test_kd.cpp:86-130: segments between random points on the bounding sphere."""
    rng = np.random.default_rng(seed)
    lo, hi = V.min(0), V.max(0)
    c = (lo + hi) / 2
    r = np.linalg.norm(hi - lo) / 2
    a = rng.normal(size=(n, 3))
    b = rng.normal(size=(n, 3))
    a = c + r * a / np.linalg.norm(a, axis=1, keepdims=True)
    b = c + r * b / np.linalg.norm(b, axis=1, keepdims=True)
    d = b - a
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = a
    rays[:, 3] = 0.0
    rays[:, 4:7] = d
    rays[:, 7] = np.inf
    return rays


def test_bunny_raycast(pg, O):
    """test_kd.cpp:86-130's protocol at the GPU trace test's bar (test_gpu_parity.py: 4,000 rays,
    >= 99.9 %): the oracle walk against a float64 Moeller-Trumbore brute force (a different triangle
    test, so only rounding-level edge cases may differ)"""
    sc, V, F = _bunny_scene(pg)
    assert len(V) == 35947 and len(F) == 69451
    osc = O.OracleScene(pg.capi, sc)
    rays = bunny_sphere_rays(V, 4000, 11)
    h = osc.trace(rays)
    prim = h[:, 1].view(np.uint32)
    t, f = _brute_force(V, F, rays[:, 0:3].astype(np.float64), rays[:, 4:7].astype(np.float64))
    hit_o = prim != 0xFFFFFFFF
    hit_b = f >= 0
    assert (hit_o == hit_b).mean() >= 0.999
    both = hit_o & hit_b
    assert both.sum() > 500
    assert (prim[both] == f[both]).mean() >= 0.999
    assert np.allclose(h[both, 0], t[both], rtol=1e-4, atol=1e-6)


def _mesh_scene(pg, V, F):
    s = pg.scenes.Scene()
    m = s.add_material(pg.scenes.material("diffuse"))
    s.add_mesh(np.ascontiguousarray(V, np.float32), np.ascontiguousarray(F, np.uint32), material=m)
    c = V.mean(0)
    s.set_camera(tuple(c + np.array([0, 0, 1.0])), tuple(c), (0, 1, 0), 40, 8, 8)
    return s.finalize()


@pytest.mark.parametrize("name", ["strip", "bunny", "ajar", "cornell", "dups"])
def test_oracle_walk_equals_brute_force(pg, O, name):
    """The oracle's BVH walk (orc_scene.h Scene::traverse: padded slab test, relative interval test,
    culling widened for ties, ties to the lower triangle index) returns exactly what a loop over every
    TriAccel returns -- the contract of the reference's kd-tree (skdtree.cpp:112-142, triaccel.h:96-157),
    which finds every hit its triangle test accepts.  The strip (triangles from x = 1 to 1.6e5) is the
    geometry on which an unpadded slab test lost 0.55 % of the hits."""
    from test_bvh4_build import geometry, rays_through
    V, F = geometry(pg, name)
    sc = pg.scenes.ajar_door(64, 36) if name == "ajar" else (
        pg.scenes.cornell(32, 32) if name == "cornell" else _mesh_scene(pg, V, F))
    osc = O.OracleScene(pg.capi, sc)
    rays = rays_through(V, F, 4000, len(F))
    rays[:, 3] = 1e-4  # the kEpsilon sentinel: the adaptive epsilon of skdtree.cpp:125-128
    walk = osc.trace(rays)
    brute = osc.trace_brute(rays)
    wp, bp = walk[:, 1].view(np.uint32), brute[:, 1].view(np.uint32)
    assert (bp != 0xFFFFFFFF).mean() > 0.2
    from test_bvh4_build import consistent_hits
    ok = consistent_hits(V, F, rays, bp, brute[:, 0])  # TriAccel hits inside their triangle's box
    assert ok.mean() > 0.995
    np.testing.assert_array_equal(wp[ok], bp[ok])
    np.testing.assert_array_equal(walk[ok, 0], brute[ok, 0])


def test_oracle_film_golden(pg, O):
    z = np.load(os.path.join(GOLDEN, "film_cornell.npz"))
    sc = pg.scenes.cornell(32, 32)
    rgbw, sq, st = O.render(O.OracleScene(pg.capi, sc), pg.capi.default_config(), 16, 0, nthreads=2)
    assert np.array_equal(st, z["stats"])
    assert np.allclose(rgbw, z["rgbw"], rtol=1e-5, atol=1e-6)
    assert np.allclose(sq, z["sumsq"], rtol=1e-5, atol=1e-6)
