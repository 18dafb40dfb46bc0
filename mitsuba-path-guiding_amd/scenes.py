"""Synthetic, seeded scene generators for the benchmark configurations:

  C1/C2  cornell()      Cornell-box class: the classic measured box, diffuse, one area light
  C3     ajar_door()    Veach ajar-door class: two rooms, door ajar ~7 deg, the only light in the far
                        room, rough-conductor + dielectric objects (~30-60k triangles)
  C4     kitchen()      Country-kitchen class interior: ~1M triangles, several area emitters
  C5     smoke()        Heterogeneous smoke: seeded fBm density grid (256^3 at full size) inside a
                        null-BSDF box, HG g = 0.8, albedo 0.9, over a diffuse floor under an area light
  (f4)   sky_courtyard()  An open courtyard lit by a procedural HDR sky envmap (sky_envmap()), the
                        environment-emitter case of SURVEY.md §8f f4

A scene is flat numpy arrays (what a Mitsuba adapter extracts from Scene::getShapes() / getBSDFs():
SURVEY.md §8b "Scene inputs it reads") plus a `desc()` that returns the pg_scene_desc for the C-ABI.
There is no network, so no Mitsuba XML scene files: these restate the scene classes procedurally.
"""
import ctypes as C

import numpy as np

from . import capi

# RGB conductor optical constants as produced by Mitsuba's spectral->RGB conversion of
# data/ior/{Cu,Al,Au}.{eta,k}.spd (roughconductor.cpp:173-188, extEta = 1 for air).
def _load_conductors():
    """RGB eta / k of the reference's conductor presets (data/ior/<name>.{eta,k}.spd through
    Spectrum::fromContinuousSpectrum, roughconductor.cpp:173-188), derived by
    tests/golden/make_conductor_fixture.py into conductors.json."""
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "conductors.json")) as f:
        mats = json.load(f)["materials"]
    return {name: (tuple(m["eta"]), tuple(m["k"])) for name, m in mats.items()}


CONDUCTORS = _load_conductors()


def _f4(v):
    v = list(v) + [0.0] * (4 - len(v))
    return capi.F4(*v[:4])


def material(kind, **kw):
    """Build a pg_material.  kind in diffuse|conductor|roughconductor|dielectric|roughdielectric|plastic|
    roughplastic|null."""
    m = capi.pg_material()
    types = {"diffuse": capi.PG_BSDF_DIFFUSE, "conductor": capi.PG_BSDF_CONDUCTOR,
             "roughconductor": capi.PG_BSDF_ROUGHCONDUCTOR, "dielectric": capi.PG_BSDF_DIELECTRIC,
             "roughdielectric": capi.PG_BSDF_ROUGHDIELECTRIC, "plastic": capi.PG_BSDF_PLASTIC,
             "roughplastic": capi.PG_BSDF_ROUGHPLASTIC, "null": capi.PG_BSDF_NULL}
    m.type = types[kind]
    dist = kw.get("distribution", "beckmann")
    m.distribution = capi.PG_DIST_GGX if dist == "ggx" else capi.PG_DIST_BECKMANN
    flags = 0
    if kw.get("twosided", False):
        flags |= capi.PG_MAT_TWOSIDED
    if kw.get("nonlinear", False):
        flags |= capi.PG_MAT_NONLINEAR
    if not kw.get("sample_visible", True):
        flags |= capi.PG_MAT_SAMPLE_ALL
    m.flags = flags
    a = kw.get("alpha", 0.1)
    m.alpha_u = kw.get("alpha_u", a)
    m.alpha_v = kw.get("alpha_v", a)
    # dielectric defaults: intIOR bk7 1.5046, extIOR air 1.000277 (dielectric.cpp); plastic polypropylene 1.49
    if kind in ("plastic", "roughplastic"):
        m.int_ior = kw.get("int_ior", 1.49)
    else:
        m.int_ior = kw.get("int_ior", 1.5046)
    m.ext_ior = kw.get("ext_ior", 1.000277)
    m.diffuse_reflectance = _f4(kw.get("reflectance", kw.get("diffuse_reflectance", (0.5, 0.5, 0.5))))
    m.specular_reflectance = _f4(kw.get("specular_reflectance", (1.0, 1.0, 1.0)))
    m.specular_transmittance = _f4(kw.get("specular_transmittance", (1.0, 1.0, 1.0)))
    if kind in ("conductor", "roughconductor"):
        name = kw.get("conductor", "Cu")
        eta, k = CONDUCTORS[name] if name != "none" else ((0, 0, 0), (1, 1, 1))
        m.eta = _f4(kw.get("eta", eta))
        m.k = _f4(kw.get("k", k))
    return m


class Scene:
    """Flat scene arrays + camera; `desc()` gives the C-ABI view (keeps arrays alive)."""

    def __init__(self):
        self._pos, self._nrm, self._idx = [], [], []
        self._nverts = 0
        self.shapes, self.materials, self.emitters = [], [], []
        self.media, self._densities = [], []
        self.camera_medium = -1
        self.camera = None
        self.envmap = None  # pg_envmap (set_envmap)
        self.mirror_x = False  # the sensor's toWorld mirrors x (mitsuba_xml): images are flipped on read-out
        self._env_rgb = None
        self._desc = None
        self.name = "scene"

    # -- construction
    def add_material(self, m):
        self.materials.append(m)
        return len(self.materials) - 1

    def add_medium(self, density, aabb_min, aabb_max, scale, albedo=(0.9, 0.9, 0.9), g=0.8):
        """Heterogeneous medium (src/medium/heterogeneous.cpp): density grid indexed [z][y][x] with
        values in [0, 1] over the data AABB, density multiplier `scale`, constant albedo, HG phase g."""
        dens = np.ascontiguousarray(density, np.float32)
        assert dens.ndim == 3
        m = capi.pg_medium()
        m.type = capi.PG_MEDIUM_HETEROGENEOUS
        m.res = (C.c_uint32 * 3)(dens.shape[2], dens.shape[1], dens.shape[0])
        m.density = dens.ctypes.data_as(C.POINTER(C.c_float))
        m.aabb_min = (C.c_float * 3)(*aabb_min)
        m.aabb_max = (C.c_float * 3)(*aabb_max)
        m.scale = scale
        m.albedo = (C.c_float * 3)(*albedo)
        m.g = g
        self._densities.append(dens)
        self.media.append(m)
        return len(self.media) - 1

    def add_mesh(self, V, F, N=None, material=0, radiance=None, interior=-1, exterior=-1):
        V = np.asarray(V, np.float32).reshape(-1, 3)
        F = np.asarray(F, np.uint32).reshape(-1, 3)
        if N is None:  # flat shading: unshare vertices, per-face normals
            tri = V[F]  # (T,3,3)
            fn = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
            fn /= np.maximum(np.linalg.norm(fn, axis=1, keepdims=True), 1e-30)
            V = tri.reshape(-1, 3)
            N = np.repeat(fn, 3, axis=0)
            F = np.arange(len(V), dtype=np.uint32).reshape(-1, 3)
        N = np.asarray(N, np.float32).reshape(-1, 3)
        tri_begin = sum(len(f) for f in self._idx)
        self._pos.append(V)
        self._nrm.append(N)
        self._idx.append(F + np.uint32(self._nverts))
        self._nverts += len(V)
        sh = capi.pg_shape(tri_begin, len(F), material, -1, interior, exterior)
        if radiance is not None:
            e = capi.pg_emitter()
            e.shape = len(self.shapes)
            e.radiance = _f4(radiance)
            self.emitters.append(e)
            sh.emitter = len(self.emitters) - 1
        self.shapes.append(sh)
        return len(self.shapes) - 1

    def set_envmap(self, rgb, to_world=None, scale=1.0):
        """Environment emitter (src/emitters/envmap.cpp): `rgb` is a latitude-longitude image of shape
        (height, width, 3), row 0 at theta = 0 (+Y of the local frame); `to_world` a 3x3 rotation."""
        rgb = np.ascontiguousarray(rgb, np.float32)
        assert rgb.ndim == 3 and rgb.shape[2] == 3
        e = capi.pg_envmap()
        e.height, e.width = rgb.shape[0], rgb.shape[1]
        e.rgb = rgb.ctypes.data_as(C.POINTER(C.c_float))
        R = np.eye(3, dtype=np.float32) if to_world is None else np.asarray(to_world, np.float32)
        e.to_world = (C.c_float * 9)(*R.reshape(-1).tolist())
        e.scale = scale
        self._env_rgb = rgb
        self.envmap = e
        self._desc = None

    def set_camera(self, origin, target, up, fov_x, width, height, near=1e-2, far=1e4):
        c = capi.pg_camera()
        c.origin = (C.c_float * 3)(*origin)
        c.target = (C.c_float * 3)(*target)
        c.up = (C.c_float * 3)(*up)
        c.fov_x_deg, c.near_clip, c.far_clip = fov_x, near, far
        c.width, c.height = width, height
        self.camera = c

    def finalize(self):
        self.positions = np.ascontiguousarray(np.concatenate(self._pos), np.float32)
        self.normals = np.ascontiguousarray(np.concatenate(self._nrm), np.float32)
        self.indices = np.ascontiguousarray(np.concatenate(self._idx), np.uint32)
        self._shapes_arr = (capi.pg_shape * len(self.shapes))(*self.shapes)
        self._mats_arr = (capi.pg_material * len(self.materials))(*self.materials)
        self._ems_arr = (capi.pg_emitter * max(1, len(self.emitters)))(*self.emitters)
        self._media_arr = (capi.pg_medium * max(1, len(self.media)))(*self.media)
        d = capi.pg_scene_desc()
        d.num_vertices = len(self.positions)
        d.num_triangles = len(self.indices)
        d.num_shapes = len(self.shapes)
        d.num_materials = len(self.materials)
        d.num_emitters = len(self.emitters)
        d.positions = self.positions.ctypes.data_as(C.POINTER(C.c_float))
        d.normals = self.normals.ctypes.data_as(C.POINTER(C.c_float))
        d.indices = self.indices.ctypes.data_as(C.POINTER(C.c_uint32))
        d.shapes = C.cast(self._shapes_arr, C.POINTER(capi.pg_shape))
        d.materials = C.cast(self._mats_arr, C.POINTER(capi.pg_material))
        d.emitters = C.cast(self._ems_arr, C.POINTER(capi.pg_emitter))
        d.camera = self.camera
        d.num_media = len(self.media)
        d.media = C.cast(self._media_arr, C.POINTER(capi.pg_medium))
        d.camera_medium = self.camera_medium
        d.envmap = C.pointer(self.envmap) if self.envmap is not None else None
        self._desc = d
        return self

    def desc(self):
        if self._desc is None:
            self.finalize()
        return self._desc

    @property
    def width(self):
        return self.camera.width

    @property
    def height(self):
        return self.camera.height

    @property
    def num_triangles(self):
        return int(sum(s.tri_count for s in self.shapes))

    def bounds(self):
        p = self.positions
        return p.min(0), p.max(0)


# ---------------------------------------------------------------------------------------------
# primitive meshes
def quad(p0, p1, p2, p3, facing=None):
    """Quad p0..p3 (CCW or CW); if `facing` is given, orient the normal toward it."""
    V = np.array([p0, p1, p2, p3], np.float32)
    F = np.array([[0, 1, 2], [0, 2, 3]], np.uint32)
    if facing is not None:
        n = np.cross(V[1] - V[0], V[2] - V[0])
        if np.dot(n, np.asarray(facing, np.float32)) < 0:
            F = F[:, ::-1].copy()
    return V, F


def box(lo, hi, inward=False):
    lo, hi = np.asarray(lo, np.float32), np.asarray(hi, np.float32)
    x0, y0, z0 = lo
    x1, y1, z1 = hi
    c = (lo + hi) / 2
    faces = [
        ((x0, y0, z0), (x1, y0, z0), (x1, y0, z1), (x0, y0, z1), (0, -1, 0)),
        ((x0, y1, z0), (x1, y1, z0), (x1, y1, z1), (x0, y1, z1), (0, 1, 0)),
        ((x0, y0, z0), (x0, y1, z0), (x0, y1, z1), (x0, y0, z1), (-1, 0, 0)),
        ((x1, y0, z0), (x1, y1, z0), (x1, y1, z1), (x1, y0, z1), (1, 0, 0)),
        ((x0, y0, z0), (x1, y0, z0), (x1, y1, z0), (x0, y1, z0), (0, 0, -1)),
        ((x0, y0, z1), (x1, y0, z1), (x1, y1, z1), (x0, y1, z1), (0, 0, 1)),
    ]
    Vs, Fs = [], []
    for a, b, cc, d, n in faces:
        n = -np.asarray(n, np.float32) if inward else np.asarray(n, np.float32)
        V, F = quad(a, b, cc, d, facing=n)
        Fs.append(F + 4 * len(Vs))
        Vs.append(V)
    return np.concatenate(Vs), np.concatenate(Fs)


def transform(V, R=None, t=(0, 0, 0), s=1.0):
    V = np.asarray(V, np.float32) * s
    if R is not None:
        V = V @ np.asarray(R, np.float32).T
    return V + np.asarray(t, np.float32)


def rot_y(deg):
    a = np.radians(deg)
    return np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]], np.float32)


def uv_sphere(center, radius, nu=64, nv=32):
    th = np.linspace(0, np.pi, nv + 1)
    ph = np.linspace(0, 2 * np.pi, nu + 1)
    T, P = np.meshgrid(th, ph, indexing="ij")
    N = np.stack([np.sin(T) * np.cos(P), np.cos(T), np.sin(T) * np.sin(P)], -1).reshape(-1, 3)
    V = N * radius + np.asarray(center, np.float32)
    F = []
    for i in range(nv):
        for j in range(nu):
            a = i * (nu + 1) + j
            b = a + nu + 1
            if i != 0:
                F.append((a, a + 1, b))
            if i != nv - 1:
                F.append((a + 1, b + 1, b))
    F = np.array(F, np.uint32)
    # orient outward
    tri = V[F]
    fn = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    if np.mean(np.sum(fn * (tri.mean(1) - np.asarray(center)), 1)) < 0:
        F = F[:, ::-1].copy()
    return V.astype(np.float32), F, N.astype(np.float32)


def torus(center, R, r, nu=96, nv=48):
    u = np.linspace(0, 2 * np.pi, nu + 1)
    v = np.linspace(0, 2 * np.pi, nv + 1)
    U, Vv = np.meshgrid(u, v, indexing="ij")
    cx, cz = np.cos(U), np.sin(U)
    N = np.stack([np.cos(Vv) * cx, np.sin(Vv), np.cos(Vv) * cz], -1).reshape(-1, 3)
    P = np.stack([(R + r * np.cos(Vv)) * cx, r * np.sin(Vv), (R + r * np.cos(Vv)) * cz], -1).reshape(-1, 3)
    P = P + np.asarray(center, np.float32)
    F = []
    for i in range(nu):
        for j in range(nv):
            a = i * (nv + 1) + j
            b = (i + 1) * (nv + 1) + j
            F.append((a, b, a + 1))
            F.append((a + 1, b, b + 1))
    F = np.array(F, np.uint32)
    tri = P[F]
    fn = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    nn = N[F].mean(1)
    if np.mean(np.sum(fn * nn, 1)) < 0:
        F = F[:, ::-1].copy()
    return P.astype(np.float32), F, N.astype(np.float32)


def cylinder(center, radius, height, n=64):
    a = np.linspace(0, 2 * np.pi, n, endpoint=False)
    c = np.asarray(center, np.float32)
    ring0 = np.stack([radius * np.cos(a), np.zeros(n), radius * np.sin(a)], -1) + c
    ring1 = ring0 + np.array([0, height, 0], np.float32)
    V = np.concatenate([ring0, ring1, [c], [c + np.array([0, height, 0])]]).astype(np.float32)
    F = []
    for i in range(n):
        j = (i + 1) % n
        F += [(i, n + i, j), (j, n + i, n + j), (2 * n, i, j), (2 * n + 1, n + j, n + i)]
    F = np.array(F, np.uint32)
    tri = V[F]
    fn = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    ctr = c + np.array([0, height / 2, 0], np.float32)
    flip = np.sum(fn * (tri.mean(1) - ctr), 1) < 0
    F[flip] = F[flip][:, ::-1]
    return V, F


# ---------------------------------------------------------------------------------------------
# C1/C2: the Cornell box (measured geometry of the Cornell data set, in metres)
def cornell(width=512, height=512, short_material=None, tall_material=None):
    """Cornell box (C1/C2).  short_material / tall_material: optional pg_material for the blocks
    (default: the white diffuse)."""
    s = Scene()
    s.name = "cornell"
    white = s.add_material(material("diffuse", reflectance=(0.725, 0.71, 0.68)))
    red = s.add_material(material("diffuse", reflectance=(0.63, 0.065, 0.05)))
    green = s.add_material(material("diffuse", reflectance=(0.14, 0.45, 0.091)))
    light = s.add_material(material("diffuse", reflectance=(0.78, 0.78, 0.78)))
    k = 0.01
    P = lambda *v: [x * k for x in v]
    inside = (278 * k, 274 * k, 280 * k)

    def wall(a, b, c, d, m):
        ctr = np.mean([a, b, c, d], 0)
        V, F = quad(a, b, c, d, facing=np.asarray(inside) - ctr)
        s.add_mesh(V, F, material=m)

    wall(P(552.8, 0, 0), P(0, 0, 0), P(0, 0, 559.2), P(549.6, 0, 559.2), white)        # floor
    wall(P(556.0, 548.8, 0), P(556.0, 548.8, 559.2), P(0, 548.8, 559.2), P(0, 548.8, 0), white)  # ceiling
    wall(P(549.6, 0, 559.2), P(0, 0, 559.2), P(0, 548.8, 559.2), P(556.0, 548.8, 559.2), white)  # back
    wall(P(0, 0, 559.2), P(0, 0, 0), P(0, 548.8, 0), P(0, 548.8, 559.2), green)       # right
    wall(P(552.8, 0, 0), P(549.6, 0, 559.2), P(556.0, 548.8, 559.2), P(556.0, 548.8, 0), red)  # left
    # light (slightly below the ceiling), facing down
    V, F = quad(P(343.0, 548.7, 227.0), P(343.0, 548.7, 332.0), P(213.0, 548.7, 332.0), P(213.0, 548.7, 227.0),
                facing=(0, -1, 0))
    s.add_mesh(V, F, material=light, radiance=(17.0, 12.0, 4.0))

    def block(quads, m):
        pts = np.array([p for q in quads for p in q], np.float32)
        ctr = pts.mean(0)
        Vs, Fs = [], []
        for q in quads:
            qc = np.mean(q, 0)
            V, F = quad(*q, facing=qc - ctr)
            Fs.append(F + 4 * len(Vs))
            Vs.append(V)
        s.add_mesh(np.concatenate(Vs), np.concatenate(Fs), material=m)

    short = [
        [P(130.0, 165.0, 65.0), P(82.0, 165.0, 225.0), P(240.0, 165.0, 272.0), P(290.0, 165.0, 114.0)],
        [P(290.0, 0.0, 114.0), P(290.0, 165.0, 114.0), P(240.0, 165.0, 272.0), P(240.0, 0.0, 272.0)],
        [P(130.0, 0.0, 65.0), P(130.0, 165.0, 65.0), P(290.0, 165.0, 114.0), P(290.0, 0.0, 114.0)],
        [P(82.0, 0.0, 225.0), P(82.0, 165.0, 225.0), P(130.0, 165.0, 65.0), P(130.0, 0.0, 65.0)],
        [P(240.0, 0.0, 272.0), P(240.0, 165.0, 272.0), P(82.0, 165.0, 225.0), P(82.0, 0.0, 225.0)],
    ]
    tall = [
        [P(423.0, 330.0, 247.0), P(265.0, 330.0, 296.0), P(314.0, 330.0, 456.0), P(472.0, 330.0, 406.0)],
        [P(423.0, 0.0, 247.0), P(423.0, 330.0, 247.0), P(472.0, 330.0, 406.0), P(472.0, 0.0, 406.0)],
        [P(472.0, 0.0, 406.0), P(472.0, 330.0, 406.0), P(314.0, 330.0, 456.0), P(314.0, 0.0, 456.0)],
        [P(314.0, 0.0, 456.0), P(314.0, 330.0, 456.0), P(265.0, 330.0, 296.0), P(265.0, 0.0, 296.0)],
        [P(265.0, 0.0, 296.0), P(265.0, 330.0, 296.0), P(423.0, 330.0, 247.0), P(423.0, 0.0, 247.0)],
    ]
    block(short, white if short_material is None else s.add_material(short_material))
    block(tall, white if tall_material is None else s.add_material(tall_material))
    s.set_camera(P(278, 273, -800), P(278, 273, -799), (0, 1, 0), 39.3077, width, height)
    return s.finalize()


# ---------------------------------------------------------------------------------------------
# C3: Veach ajar-door class.  Room A (camera) x in [0,5], room B (light) x in [5.15, 9];
# y up in [0, 3]; z in [0, 5].  Doorway in the separating wall at z in [2.0, 3.0], y < 2.2; the
# door is hinged at (5.0, z=2.0) and opened by `door_deg` into room A: light reaches room A only
# through the narrow gap.  The only emitter is a ceiling panel in room B.
def ajar_door(width=1280, height=720, door_deg=7.0, sphere_res=(96, 48), seed=7, diffuse_objects=False):
    """diffuse_objects: the table, spheres, torus and pebbles diffuse (grey 0.5) instead of rough
    metals and glass -- the camera room is then lit only indirectly, without specular chains."""
    rng = np.random.default_rng(seed)
    s = Scene()
    s.name = "ajar_diffuse" if diffuse_objects else "ajar_door"
    wallm = s.add_material(material("diffuse", reflectance=(0.6, 0.58, 0.55)))
    floorm = s.add_material(material("diffuse", reflectance=(0.35, 0.28, 0.22)))
    doorm = s.add_material(material("diffuse", reflectance=(0.45, 0.40, 0.35), twosided=True))
    tablem = s.add_material(material("roughconductor", conductor="Al", alpha=0.2, distribution="ggx"))
    cu = s.add_material(material("roughconductor", conductor="Cu", alpha=0.05, distribution="ggx"))
    au = s.add_material(material("roughconductor", conductor="Au", alpha=0.4, distribution="beckmann"))
    glass = s.add_material(material("dielectric", int_ior=1.5, ext_ior=1.0))
    rglass = s.add_material(material("roughdielectric", int_ior=1.5, ext_ior=1.0, alpha=0.2, distribution="ggx"))
    lightm = s.add_material(material("diffuse", reflectance=(0.0, 0.0, 0.0)))
    if diffuse_objects:
        tablem = cu = au = glass = rglass = s.add_material(material("diffuse", reflectance=(0.5, 0.5, 0.5)))
    H = 3.0
    xa, xw, xb, Z = 5.0, 5.15, 9.0, 5.0
    ins_a = (2.5, 1.5, 2.5)
    ins_b = (7.0, 1.5, 2.5)

    def wall(a, b, c, d, m, toward):
        ctr = np.mean([a, b, c, d], 0)
        V, F = quad(a, b, c, d, facing=np.asarray(toward) - ctr)
        s.add_mesh(V, F, material=m)

    # room A shell
    wall((0, 0, 0), (xa, 0, 0), (xa, 0, Z), (0, 0, Z), floorm, ins_a)
    wall((0, H, 0), (xa, H, 0), (xa, H, Z), (0, H, Z), wallm, ins_a)
    wall((0, 0, 0), (0, H, 0), (0, H, Z), (0, 0, Z), wallm, ins_a)
    wall((0, 0, 0), (xa, 0, 0), (xa, H, 0), (0, H, 0), wallm, ins_a)
    wall((0, 0, Z), (xa, 0, Z), (xa, H, Z), (0, H, Z), wallm, ins_a)
    # room B shell
    wall((xw, 0, 0), (xb, 0, 0), (xb, 0, Z), (xw, 0, Z), floorm, ins_b)
    wall((xw, H, 0), (xb, H, 0), (xb, H, Z), (xw, H, Z), wallm, ins_b)
    wall((xb, 0, 0), (xb, H, 0), (xb, H, Z), (xb, 0, Z), wallm, ins_b)
    wall((xw, 0, 0), (xb, 0, 0), (xb, H, 0), (xw, H, 0), wallm, ins_b)
    wall((xw, 0, Z), (xb, 0, Z), (xb, H, Z), (xw, H, Z), wallm, ins_b)
    # separating wall with a doorway (z in [2,3], y in [0,2.2]): faces on both sides + jambs
    z0, z1, yd = 2.0, 3.0, 2.2
    for x, toward in ((xa, ins_a), (xw, ins_b)):
        wall((x, 0, 0), (x, H, 0), (x, H, z0), (x, 0, z0), wallm, toward)
        wall((x, 0, z1), (x, H, z1), (x, H, Z), (x, 0, Z), wallm, toward)
        wall((x, yd, z0), (x, H, z0), (x, H, z1), (x, yd, z1), wallm, toward)
    wall((xa, 0, z0), (xw, 0, z0), (xw, yd, z0), (xa, yd, z0), wallm, (xa, 1, 2.5))
    wall((xa, 0, z1), (xw, 0, z1), (xw, yd, z1), (xa, yd, z1), wallm, (xa, 1, 2.5))
    wall((xa, yd, z0), (xw, yd, z0), (xw, yd, z1), (xa, yd, z1), wallm, (xa, 1, 2.5))
    # the door: 0.05 thick slab hinged at (xa, z0), rotated into room A by door_deg
    V, F = box((0.0, 0.0, 0.0), (0.05, yd - 0.01, (z1 - z0) - 0.01))
    V = transform(V - np.array([0.05, 0, 0], np.float32), R=rot_y(door_deg), t=(xa, 0.0, z0 + 0.005))
    s.add_mesh(V, F, material=doorm)
    # the light: ceiling panel in room B, facing down
    V, F = quad((6.5, H - 0.01, 1.5), (8.5, H - 0.01, 1.5), (8.5, H - 0.01, 3.5), (6.5, H - 0.01, 3.5),
                facing=(0, -1, 0))
    s.add_mesh(V, F, material=lightm, radiance=(40.0, 36.0, 30.0))
    # furniture in room A: a table (aluminium top, legs) with objects
    V, F = box((1.2, 0.75, 1.4), (3.4, 0.8, 3.4))
    s.add_mesh(V, F, material=tablem)
    for (lx, lz) in ((1.3, 1.5), (3.3, 1.5), (1.3, 3.3), (3.3, 3.3)):
        V, F = box((lx - 0.04, 0.0, lz - 0.04), (lx + 0.04, 0.75, lz + 0.04))
        s.add_mesh(V, F, material=tablem)
    nu, nv = sphere_res
    V, F, N = uv_sphere((1.8, 0.8 + 0.25, 2.0), 0.25, nu, nv)
    s.add_mesh(V, F, N, material=cu)
    V, F, N = uv_sphere((2.6, 0.8 + 0.2, 2.9), 0.2, nu, nv)
    s.add_mesh(V, F, N, material=glass)
    V, F, N = uv_sphere((2.9, 0.8 + 0.15, 1.9), 0.15, nu, nv)
    s.add_mesh(V, F, N, material=au)
    V, F, N = torus((2.1, 0.8 + 0.08, 3.0), 0.22, 0.08, 2 * nu, nv)
    s.add_mesh(V, F, N, material=rglass)
    # a few random pebbles on the floor (seeded)
    for i in range(6):
        c = (rng.uniform(0.5, 4.5), 0.1, rng.uniform(0.5, 4.5))
        V, F, N = uv_sphere(c, 0.1, nu // 2, nv // 2)
        s.add_mesh(V, F, N, material=[cu, au, rglass][i % 3])
    s.set_camera((0.3, 1.6, 0.4), (4.0, 1.0, 2.8), (0, 1, 0), 65.0, width, height)
    return s.finalize()


# ---------------------------------------------------------------------------------------------
# C4: country-kitchen class interior, ~1M triangles, several area emitters
def kitchen(width=1920, height=1080, target_tris=1_000_000, seed=7):
    rng = np.random.default_rng(seed)
    s = Scene()
    s.name = "kitchen"
    wall = s.add_material(material("diffuse", reflectance=(0.7, 0.66, 0.6)))
    wood = s.add_material(material("diffuse", reflectance=(0.45, 0.3, 0.18)))
    tile = s.add_material(material("plastic", diffuse_reflectance=(0.5, 0.5, 0.45)))
    steel = s.add_material(material("roughconductor", conductor="Al", alpha=0.15, distribution="ggx"))
    copper = s.add_material(material("roughconductor", conductor="Cu", alpha=0.3, distribution="ggx"))
    ceramic = s.add_material(material("plastic", diffuse_reflectance=(0.8, 0.78, 0.7)))
    glass = s.add_material(material("dielectric", int_ior=1.5, ext_ior=1.0))
    lm = s.add_material(material("diffuse", reflectance=(0, 0, 0)))
    W, Hh, D = 6.0, 3.0, 5.0
    V, F = box((0, 0, 0), (W, Hh, D), inward=True)
    s.add_mesh(V, F, material=wall)
    V, F = quad((0, 0.001, 0), (W, 0.001, 0), (W, 0.001, D), (0, 0.001, D), facing=(0, 1, 0))
    s.add_mesh(V, F, material=tile)
    # counters and cabinets along the back wall
    for i in range(6):
        x0 = 0.2 + i * 0.95
        V, F = box((x0, 0, D - 0.65), (x0 + 0.9, 0.9, D - 0.05))
        s.add_mesh(V, F, material=wood)
        V, F = box((x0, 1.6, D - 0.4), (x0 + 0.9, 2.4, D - 0.05))
        s.add_mesh(V, F, material=wood)
    V, F = box((0.2, 0.9, D - 0.68), (5.9, 0.95, D - 0.02))
    s.add_mesh(V, F, material=steel)
    # table
    V, F = box((2.0, 0.75, 1.8), (4.0, 0.8, 3.0))
    s.add_mesh(V, F, material=wood)
    for (lx, lz) in ((2.1, 1.9), (3.9, 1.9), (2.1, 2.9), (3.9, 2.9)):
        V, F = box((lx - 0.04, 0, lz - 0.04), (lx + 0.04, 0.75, lz + 0.04))
        s.add_mesh(V, F, material=wood)
    # lights: 4 ceiling panels + one window panel
    for (cx, cz) in ((1.5, 1.5), (4.5, 1.5), (1.5, 3.5), (4.5, 3.5)):
        V, F = quad((cx - 0.3, Hh - 0.01, cz - 0.3), (cx + 0.3, Hh - 0.01, cz - 0.3), (cx + 0.3, Hh - 0.01, cz + 0.3),
                    (cx - 0.3, Hh - 0.01, cz + 0.3), facing=(0, -1, 0))
        s.add_mesh(V, F, material=lm, radiance=(12.0, 11.0, 9.0))
    V, F = quad((0.01, 1.0, 1.5), (0.01, 2.2, 1.5), (0.01, 2.2, 3.0), (0.01, 1.0, 3.0), facing=(1, 0, 0))
    s.add_mesh(V, F, material=lm, radiance=(6.0, 7.0, 9.0))
    # clutter: spheres / tori / cylinders on counters, table and shelves until ~target_tris
    mats = [steel, copper, ceramic, glass, wood]
    placements = []
    for _ in range(4000):
        r = rng.random()
        if r < 0.4:
            placements.append((rng.uniform(2.1, 3.9), 0.8, rng.uniform(1.9, 2.9)))
        elif r < 0.8:
            placements.append((rng.uniform(0.3, 5.8), 0.95, rng.uniform(D - 0.6, D - 0.1)))
        else:
            placements.append((rng.uniform(0.3, 5.8), 2.4, rng.uniform(D - 0.38, D - 0.08)))
    k = 0
    while s.num_triangles < target_tris and k < len(placements):
        x, y, z = placements[k]
        m = mats[k % len(mats)]
        kind = k % 3
        if kind == 0:
            rad = rng.uniform(0.03, 0.07)
            V, F, N = uv_sphere((x, y + rad, z), rad, 64, 32)
            s.add_mesh(V, F, N, material=m)
        elif kind == 1:
            V, F, N = torus((x, y + 0.02, z), 0.05, 0.02, 64, 32)
            s.add_mesh(V, F, N, material=m)
        else:
            V, F = cylinder((x, y, z), rng.uniform(0.02, 0.05), rng.uniform(0.08, 0.25), 48)
            s.add_mesh(V, F, material=m)
        k += 1
    s.set_camera((0.5, 1.7, 0.3), (3.5, 1.0, 4.0), (0, 1, 0), 70.0, width, height)
    return s.finalize()


# ---------------------------------------------------------------------------------------------
# C5: heterogeneous smoke
# ---------------------------------------------------------------------------------------------
# environment-lit scenes (the envmap emitter of data/tests/test_emitter.xml)
def rot_x(deg):
    a = np.radians(deg)
    return np.array([[1, 0, 0], [0, np.cos(a), -np.sin(a)], [0, np.sin(a), np.cos(a)]], np.float32)


def sky_envmap(width=256, height=128, sun_theta=40.0, sun_phi=60.0, sun_radius=3.0, sun_radiance=400.0, seed=7):
    """Procedural latitude-longitude sky (seeded): a zenith-to-horizon gradient, a dim ground half with
    a little noise, and a small bright sun disk, i.e. the high-dynamic-range, strongly peaked kind of
    map guiding and envmap importance sampling are for.  Returns (height, width, 3) float32."""
    rng = np.random.default_rng(seed)
    th = (np.arange(height) + 0.5) / height * np.pi
    ph = (np.arange(width) + 0.5) / width * 2 * np.pi
    T, P = np.meshgrid(th, ph, indexing="ij")
    img = np.zeros((height, width, 3), np.float32)
    up = np.cos(T)
    sky = np.stack([0.35 + 0.4 * (1 - up), 0.55 + 0.3 * (1 - up), 0.95 + 0.05 * up], -1) * (up > 0)[..., None]
    ground = np.stack([0.12, 0.1, 0.08], -1) * (up <= 0)[..., None] * (0.8 + 0.4 * rng.random((height, width, 1)))
    img += sky + ground
    # local direction (envmap.cpp:598): (sin phi sin theta, cos theta, -cos phi sin theta)
    d = np.stack([np.sin(P) * np.sin(T), np.cos(T), -np.cos(P) * np.sin(T)], -1)
    st, sp = np.radians(sun_theta), np.radians(sun_phi)
    sd = np.array([np.sin(sp) * np.sin(st), np.cos(st), -np.cos(sp) * np.sin(st)])
    ang = np.degrees(np.arccos(np.clip(d @ sd, -1, 1)))
    img += (ang < sun_radius)[..., None] * np.array([1.0, 0.9, 0.75], np.float32) * sun_radiance
    return img.astype(np.float32)


def sky_courtyard(width=512, height=384, seed=7, env=None, area_light=False):
    """An open courtyard under a sky envmap: a ground plane, walls that shade part of it, and
    diffuse / rough-conductor / glass / plastic objects (optionally one area light).  Light reaches
    most shading points only through the environment emitter."""
    rng = np.random.default_rng(seed)
    s = Scene()
    s.name = "sky_courtyard"
    ground = s.add_material(material("diffuse", reflectance=(0.45, 0.42, 0.38)))
    wall = s.add_material(material("diffuse", reflectance=(0.7, 0.65, 0.6), twosided=True))
    gold = s.add_material(material("roughconductor", conductor="Au", alpha=0.2, distribution="ggx"))
    glass = s.add_material(material("roughdielectric", int_ior=1.5, ext_ior=1.0, alpha=0.1, distribution="ggx"))
    red = s.add_material(material("roughplastic", alpha=0.3, distribution="ggx", diffuse_reflectance=(0.6, 0.15, 0.1)))
    V, F = quad((-6, 0, -6), (6, 0, -6), (6, 0, 6), (-6, 0, 6), facing=(0, 1, 0))
    s.add_mesh(V, F, material=ground)
    V, F = box((-4, 0, 2.5), (4, 2.5, 2.8))
    s.add_mesh(V, F, material=wall)
    V, F = box((2.5, 0, -3), (2.8, 2.0, 2.5))
    s.add_mesh(V, F, material=wall)
    V, F, N = uv_sphere((-1.0, 0.8, 0.5), 0.8, 64, 32)
    s.add_mesh(V, F, N, material=gold)
    V, F, N = uv_sphere((0.9, 0.6, -0.4), 0.6, 64, 32)
    s.add_mesh(V, F, N, material=glass)
    V, F = box((-0.3, 0, -1.8), (0.5, 0.9, -1.0))
    s.add_mesh(transform(V, rot_y(25), t=(0, 0, 0)), F, material=red)
    for i in range(5):
        c = (rng.uniform(-3, 2), 0.15, rng.uniform(-3, 2))
        V, F, N = uv_sphere(c, 0.15, 24, 12)
        s.add_mesh(V, F, N, material=[gold, red, ground][i % 3])
    if area_light:
        lm = s.add_material(material("diffuse", reflectance=(0, 0, 0)))
        V, F = quad((1.5, 2.4, 1.5), (2.3, 2.4, 1.5), (2.3, 2.4, 2.3), (1.5, 2.4, 2.3), facing=(0, -1, 0))
        s.add_mesh(V, F, material=lm, radiance=(8.0, 7.0, 6.0))
    s.set_envmap(sky_envmap(seed=seed) if env is None else env, to_world=rot_y(0))
    s.set_camera((-4.5, 2.2, -5.5), (0.2, 0.6, 0.3), (0, 1, 0), 60.0, width, height)
    return s.finalize()


def fbm_density(res=256, seed=7, octaves=5, base=4):
    """Seeded fBm density in [0, 1] on a res^3 grid ([z][y][x]): value-noise octaves (trilinear
    upsampling of random lattices, base * 2^o cells per axis, amplitude 2^-o) shaped by a soft
    spherical falloff and a threshold, so the cloud has empty space, wisps and a dense core."""
    rng = np.random.default_rng(seed)
    x = (np.arange(res, dtype=np.float32) + 0.5) / res  # cell-centred coordinates in (0, 1)
    acc = np.zeros((res, res, res), np.float32)
    amp, total = 1.0, 0.0
    for o in range(octaves):
        n = base * (2 ** o)
        lat = rng.random((n + 1, n + 1, n + 1), dtype=np.float32)
        f = x * n
        i0 = np.minimum(f.astype(np.int32), n - 1)
        w = (f - i0).astype(np.float32)
        w = w * w * (3 - 2 * w)  # smoothstep fade
        # separable trilinear interpolation: z, then y, then x
        a = lat[i0] * (1 - w)[:, None, None] + lat[i0 + 1] * w[:, None, None]              # (res, n+1, n+1)
        a = a[:, i0] * (1 - w)[None, :, None] + a[:, i0 + 1] * w[None, :, None]            # (res, res, n+1)
        a = a[:, :, i0] * (1 - w)[None, None, :] + a[:, :, i0 + 1] * w[None, None, :]      # (res, res, res)
        acc += amp * a
        total += amp
        amp *= 0.5
        del a
    acc /= total
    c = x - 0.5
    r2 = c[:, None, None] ** 2 + c[None, :, None] ** 2 + c[None, None, :] ** 2
    shape = np.clip(1.0 - r2 / 0.22, 0.0, 1.0)
    d = np.clip((acc * shape - 0.18) * 2.5, 0.0, 1.0).astype(np.float32)
    return d


def smoke(width=1024, height=1024, res=256, seed=7, scale=40.0, albedo=0.9, g=0.8):
    """C5: the smoke cloud (fBm grid over [-1, 1]^3, enclosed by a null-BSDF box whose interior is
    the medium) above a diffuse floor, lit by one area light; camera outside the medium."""
    s = Scene()
    s.name = "smoke"
    floor = s.add_material(material("diffuse", reflectance=(0.6, 0.6, 0.6)))
    lightm = s.add_material(material("diffuse", reflectance=(0.0, 0.0, 0.0)))
    nullm = s.add_material(material("null"))
    dens = fbm_density(res, seed)
    med = s.add_medium(dens, (-1.0, -1.0, -1.0), (1.0, 1.0, 1.0), scale, (albedo, albedo, albedo), g)
    V, F = box((-1.0, -1.0, -1.0), (1.0, 1.0, 1.0))  # outward normals: interior = inside the box
    s.add_mesh(V, F, material=nullm, interior=med)
    V, F = quad((-6, -1.2, -6), (6, -1.2, -6), (6, -1.2, 6), (-6, -1.2, 6), facing=(0, 1, 0))
    s.add_mesh(V, F, material=floor)
    V, F = quad((-1.5, 4.0, -2.5), (1.5, 4.0, -2.5), (1.5, 3.0, -0.5), (-1.5, 3.0, -0.5), facing=(0, -1, 0.5))
    s.add_mesh(V, F, material=lightm, radiance=(30.0, 28.0, 24.0))
    s.set_camera((0.0, 0.6, 4.2), (0.0, -0.1, 0.0), (0, 1, 0), 45.0, width, height)
    return s.finalize()


SCENES = {"cornell": cornell, "ajar_door": ajar_door,
          "ajar_diffuse": lambda w=1280, h=720: ajar_door(w, h, diffuse_objects=True), "kitchen": kitchen, "smoke": smoke, "sky_courtyard": sky_courtyard}
