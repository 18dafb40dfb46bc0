"""The library's closest-hit BVH (pg_bvh.cpp, 4-wide nodes of pg_layout.h PG_QNODE_*) built and walked
on the CPU through a test-only shim (tests/csrc/bvh_shim.cpp): every triangle sits in exactly one
leaf, every child box contains its subtree, the stack bound the builder checks holds, and a scalar
restatement of the device walk (traverse4) returns exactly the brute-force closest hit over the same
triangle records (TriAccel; bit-exact t and triangle, lower index on ties) -- on the C3 and Cornell scenes, the
bunny of data/tests/bunny.ply, coplanar duplicates and a geometric progression that drives the binned
SAH build into its deepest trees.  The GPU walk is checked against the oracle in test_gpu_parity."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
QSTACK_DEPTH = 96  # pg_layout.h PG_QSTACK_DEPTH


SHIM_SOURCES = [os.path.join(ROOT, "tests", "csrc", "bvh_shim.cpp"),
                os.path.join(ROOT, "mitsuba-path-guiding_amd", "csrc", "pg_bvh.cpp"),
                os.path.join(ROOT, "mitsuba-path-guiding_amd", "csrc", "pg_layout.h")]
PREBUILT = os.path.join(ROOT, "tests", "csrc", "_build", "libbvhshim.so")  # __graft_entry__.build()
# the same shim with FMA contraction (A/B of the Woop records, PG_TRIACCEL = 0, whose device test contracts)
PREBUILT_FMA = os.path.join(ROOT, "tests", "csrc", "_build", "libbvhshim_fma.so")


def compile_shim(out, fma=False):
    contract = ["-ffp-contract=fast", "-mfma"] if fma else ["-ffp-contract=off"]
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", *contract, "-o", out, *SHIM_SOURCES[:2]])


def build_shim(tmp_path_factory, fma=False):
    out = PREBUILT_FMA if fma else PREBUILT
    if not os.path.exists(out) or any(os.path.getmtime(f) > os.path.getmtime(out) for f in SHIM_SOURCES):
        out = str(tmp_path_factory.mktemp("bvhshim") / ("libbvhshim_fma.so" if fma else "libbvhshim.so"))
        compile_shim(out, fma)
    L = C.CDLL(out)
    L.shim_build.restype = C.c_int
    L.shim_build.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]
    L.shim_check.argtypes = [C.c_uint32, C.c_void_p]
    L.shim_trace.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint32]
    L.shim_order.argtypes = [C.c_void_p]
    return L


@pytest.fixture(scope="module")
def shim(tmp_path_factory):
    return build_shim(tmp_path_factory)


def brute_force_hits(shim, V, F, rays, with_t=False):
    """original triangle id (or ~0) of the closest hit of every ray, by brute force over the library's
    triangle records (the shim's loop)"""
    V, F = np.ascontiguousarray(V, np.float32), np.ascontiguousarray(F, np.uint32)
    assert shim.shim_build(V.ctypes.data, len(V), F.ctypes.data, len(F)) == 1
    n = len(rays)
    walk = np.zeros((n, 2), np.uint32)
    brute = np.zeros((n, 2), np.uint32)
    shim.shim_trace(np.ascontiguousarray(rays).ctypes.data, n, walk.ctypes.data, brute.ctypes.data, len(F))
    order = np.zeros(len(F), np.uint32)
    shim.shim_order(order.ctypes.data)
    hit = brute[:, 1] != 0xFFFFFFFF
    out = np.full(n, 0xFFFFFFFF, np.uint32)
    out[hit] = order[brute[hit, 1]]
    return (out, brute[:, 0].view(np.float32).copy()) if with_t else out


def consistent_hits(V, F, rays, prim, t):
    """Rays whose hit distance t lies in the slab interval of the hit triangle's bounding box, widened by
    half the walks' own padding (2^-22 max_a |o_a / d_a| + 2^-22 t; pg_trace.h slabRay pads by 2^-21).
    A grazing ray far from the origin can make the fp32 triangle test (the reference's TriAccel
    included) report a t off by ~100 ulps, i.e. a hit outside the triangle's own box: no box walk can be
    required to find those (the reference's kd-tree clips its leaves too).  Misses count as consistent."""
    ok = np.ones(len(rays), bool)
    h = prim != 0xFFFFFFFF
    P = V[F[prim[h]]].astype(np.float64)
    o, d = rays[h, 0:3].astype(np.float64), rays[h, 4:7].astype(np.float64)
    d = np.where(np.abs(d) > 1e-30, d, 1e-30)
    ta, tb = (P.min(1) - o) / d, (P.max(1) - o) / d
    t0, t1 = np.minimum(ta, tb).max(1), np.maximum(ta, tb).min(1)
    th = t[h].astype(np.float64)
    pad = 2.0 ** -22 * (np.abs(o / d).max(1) + np.abs(th))
    ok[h] = (th >= t0 - pad) & (th <= t1 + pad)
    return ok


def geometric_strip(n=3000):
    """triangles at x = 1.004^k: centroid bins stay lopsided, so the SAH build peels a few triangles per
    level down to its depth-32 median fallback"""
    x = 1.004 ** np.arange(n, dtype=np.float64)
    V = np.zeros((3 * n, 3), np.float32)
    V[0::3, 0], V[1::3, 0], V[2::3, 0] = x, x + 0.01 * x, x
    V[1::3, 1], V[2::3, 2] = 0.01 * x, 0.01 * x
    return V, np.arange(3 * n, dtype=np.uint32).reshape(n, 3)


def coplanar_duplicates(n=500, seed=3):
    """every triangle twice (ties at equal t) plus a shared-edge fan"""
    rng = np.random.default_rng(seed)
    V = rng.random((3 * n, 3)).astype(np.float32)
    F = np.arange(3 * n, dtype=np.uint32).reshape(n, 3)
    return V, np.concatenate([F, F[::-1]])


def geometry(pg, name):
    if name == "bunny":
        z = np.load(os.path.join(ROOT, "tests", "golden", "bunny.npz"))
        return z["positions"].astype(np.float32), z["faces"].astype(np.uint32)
    if name == "strip":
        return geometric_strip()
    if name == "dups":
        return coplanar_duplicates()
    if name == "single":
        return np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32), np.array([[0, 1, 2]], np.uint32)
    sc = pg.scenes.ajar_door(64, 36) if name == "ajar" else pg.scenes.cornell(32, 32)
    return sc.positions.reshape(-1, 3), sc.indices.reshape(-1, 3)


def rays_through(V, F, n, seed):
    rng = np.random.default_rng(seed)
    lo, hi = V.min(0), V.max(0)
    ctr, rad = (lo + hi) / 2, np.linalg.norm(hi - lo) / 2 + 1e-3
    a = rng.normal(size=(n, 3))
    a = ctr + rad * 1.2 * a / np.linalg.norm(a, axis=1, keepdims=True)
    b = V[F[rng.integers(0, len(F), n)]].mean(1)  # aimed at triangle centroids
    d = (b - a) / np.linalg.norm(b - a, axis=1, keepdims=True)
    inner = rng.random(n) < 0.5  # half the rays start inside the scene
    a[inner] = (lo + (hi - lo) * rng.random((n, 3)))[inner]
    r = np.zeros((n, 8), np.float32)
    r[:, 0:3], r[:, 3], r[:, 4:7], r[:, 7] = a, 1e-5, d, np.inf
    return r


@pytest.mark.parametrize("name", ["ajar", "cornell", "bunny", "strip", "dups", "single"])
def test_bvh4_structure_and_walk(pg, shim, name):
    V, F = geometry(pg, name)
    V, F = np.ascontiguousarray(V, np.float32), np.ascontiguousarray(F, np.uint32)
    nt = len(F)
    assert shim.shim_build(V.ctypes.data, len(V), F.ctypes.data, nt) == 1
    info = np.zeros(5, np.uint32)
    shim.shim_check(nt, info.ctypes.data)
    nodes, need, once, bad, depth = (int(x) for x in info)
    assert once == nt, "every triangle in exactly one leaf"
    assert bad == 0, "child boxes contain their subtrees"
    assert need <= QSTACK_DEPTH
    if name == "strip":
        assert need > 16  # the walk spills past the LDS stack into the overflow ring on this tree
    n = 2000 if nt > 20000 else 4000
    rays = rays_through(V, F, n, nt)
    walk = np.zeros((n, 2), np.uint32)
    brute = np.zeros((n, 2), np.uint32)
    shim.shim_trace(rays.ctypes.data, n, walk.ctypes.data, brute.ctypes.data, nt)
    assert (brute[:, 1] != 0xFFFFFFFF).mean() > (0.0 if name == "single" else 0.2)
    np.testing.assert_array_equal(walk, brute)


@pytest.mark.parametrize("name", ["ajar", "cornell", "bunny", "strip"])
def test_triangle_records_equal_oracle_triaccel(pg, O, shim, name):
    """The library's triangle records are the reference's TriAccel built in fp32 (pg_bvh.cpp
    triAccelRecord, triaccel.h:37-94), tested without contraction: over the same rays the library's
    walk and the oracle's (its own BVH, orc_scene.h TriAccel) return the same triangle and the same t
    bit for bit (ties aside: the library breaks them by BVH order, the oracle by original index)."""
    V, F = geometry(pg, name)
    V, F = np.ascontiguousarray(V, np.float32), np.ascontiguousarray(F, np.uint32)
    nt = len(F)
    assert shim.shim_build(V.ctypes.data, len(V), F.ctypes.data, nt) == 1
    n = 2000 if nt > 20000 else 4000
    rays = rays_through(V, F, n, nt + 1)  # tmin 1e-5 on both sides (not the 1e-4 adaptive-epsilon sentinel)
    walk = np.zeros((n, 2), np.uint32)
    brute = np.zeros((n, 2), np.uint32)
    shim.shim_trace(rays.ctypes.data, n, walk.ctypes.data, brute.ctypes.data, nt)
    order = np.zeros(nt, np.uint32)
    shim.shim_order(order.ctypes.data)
    lib = np.full(n, 0xFFFFFFFF, np.uint32)
    hit = walk[:, 1] != 0xFFFFFFFF
    lib[hit] = order[walk[hit, 1]]
    s = pg.scenes.Scene()
    s.add_mesh(V, F, material=s.add_material(pg.scenes.material("diffuse")))
    s.set_camera(tuple(V.mean(0) + np.array([0, 0, 1.0])), tuple(V.mean(0)), (0, 1, 0), 40, 8, 8)
    osc = O.OracleScene(pg.capi, s.finalize())
    c = osc.trace(rays)
    cp = c[:, 1].view(np.uint32)
    assert (lib != 0xFFFFFFFF).mean() > 0.2
    ok = consistent_hits(V, F, rays, cp, c[:, 0])
    assert ok.mean() > 0.99
    same = lib == cp
    assert same[ok].mean() >= 0.995, same[ok].mean()  # ties: BVH order here, original index in the oracle
    both = same & hit
    np.testing.assert_array_equal(walk[both, 0].view(np.float32), c[both, 0])
