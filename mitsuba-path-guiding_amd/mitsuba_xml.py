"""Mitsuba 0.5 XML scene subset -> Scene ("XML scene subset loader").

The reference parses scenes with Xerces into Properties and plugin objects
(src/librender/scenehandler.cpp, data/schema/scene.xsd, doc/format.tex).  This module reads the
subset the MI355X path renders and flattens it straight into a `scenes.Scene`, i.e. what a Mitsuba
adapter's flatten() produces from Scene::getShapes()/getBSDFs():

  scene structure   <scene>, <default name value>, $name substitution, id / <ref id>
  properties        float, integer, boolean, string, rgb, srgb, spectrum (single value), point, vector
  transforms        translate, rotate (axis + degrees), scale, matrix (row-major 4x4), lookat
                    (Transform::translate/rotate/scale/lookAt, src/libcore/transform.cpp)
  integrator        any type: (type, properties) returned for the caller (ProgressivePathTracer props)
  sensor            perspective: fov, fovAxis (x, y, diagonal, smaller, larger), nearClip, farClip,
                    toWorld (a mirrored camera, e.g. <scale x="-1"/>, sets Scene.mirror_x);
                    sampler sampleCount; film width / height (the filter is always the 1-px box)
  bsdf              diffuse, conductor, roughconductor (material Cu / Al / Au / none, or eta + k),
                    dielectric, roughdielectric, plastic, roughplastic (intIOR / extIOR by value or
                    by name: src/bsdfs/ior.h), twosided, null; distribution beckmann / ggx
  shape             obj, ply (ascii / binary), serialized (Mitsuba's zlib mesh format, any shapeIndex),
                    rectangle, cube, disk and sphere (tessellated), with
                    toWorld, flipNormals, faceNormals, a nested or referenced bsdf and an area emitter
  emitter           area (in a shape), envmap (.npy / .pfm / uncompressed or zlib EXR), constant
                    (as a uniform envmap)
  medium            homogeneous (sigmaS / sigmaA or sigmaT / albedo, scale, g; grey sigmaT) with an hg or
                    isotropic phase, declared at the top level or nested in a shape, attached to
                    shapes as <ref name="interior|exterior">; a shape without a BSDF is a null
                    (index-matched) surface when it is a medium transition, black diffuse when it is
                    an emitter, 0.5 diffuse otherwise (Shape::configure, shape.cpp:48-72)

Anything else raises NotImplementedError naming the plugin (strict=True), or is collected in
`XMLScene.skipped` (strict=False).  Mesh normals follow TriMesh::computeNormals (trimesh.cpp:608-680):
a mesh without normals gets angle-weighted vertex normals unless faceNormals is set.
"""
import math
import os
import re
import struct
import xml.etree.ElementTree as ET
import zlib

import numpy as np

from . import capi, scenes

# src/bsdfs/ior.h:39-64
IOR = {"vacuum": 1.0, "helium": 1.000036, "hydrogen": 1.000132, "air": 1.000277, "carbon dioxide": 1.00045,
       "water": 1.3330, "acetone": 1.36, "ethanol": 1.361, "carbon tetrachloride": 1.461, "glycerol": 1.4729,
       "benzene": 1.501, "silicone oil": 1.52045, "bromine": 1.661, "water ice": 1.31, "fused quartz": 1.458,
       "pyrex": 1.470, "acrylic glass": 1.49, "polypropylene": 1.49, "bk7": 1.5046, "sodium chloride": 1.544,
       "amber": 1.55, "pet": 1.5750, "diamond": 2.419}


class XMLScene:
    """Result of load(): the finalized Scene, the integrator (type, props) and the sampler's spp."""

    def __init__(self):
        self.scene = None
        self.integrator_type = None
        self.integrator_props = {}
        self.spp = None
        self.bsdfs = []      # (id or type, pg_material) of every top-level BSDF, in file order
        self.skipped = []    # (tag, type, reason) when strict=False


def _floats(s):
    return [float(x) for x in re.split(r"[,\s]+", s.strip()) if x]


def _srgb_to_linear(c):
    c = np.asarray(c, np.float64)
    return np.where(c <= 0.04045, c / 12.92, ((c + 0.055) / 1.055) ** 2.4)


# ---- transforms (src/libcore/transform.cpp) ---------------------------------------------------
def _rotate(axis, deg):
    a = np.asarray(axis, np.float64)
    a = a / np.linalg.norm(a)
    s, c = math.sin(math.radians(deg)), math.cos(math.radians(deg))
    x, y, z = a
    M = np.eye(4)
    M[:3, :3] = [[x * x + (1 - x * x) * c, x * y * (1 - c) - z * s, x * z * (1 - c) + y * s],
                 [x * y * (1 - c) + z * s, y * y + (1 - y * y) * c, y * z * (1 - c) - x * s],
                 [x * z * (1 - c) - y * s, y * z * (1 - c) + x * s, z * z + (1 - z * z) * c]]
    return M


def _lookat(origin, target, up):
    o, t, u = (np.asarray(v, np.float64) for v in (origin, target, up))
    d = (t - o) / np.linalg.norm(t - o)
    left = np.cross(u, d)
    left /= np.linalg.norm(left)
    nup = np.cross(d, left)
    M = np.eye(4)
    M[:3, 0], M[:3, 1], M[:3, 2], M[:3, 3] = left, nup, d, o
    return M


class _Loader:
    def __init__(self, base_dir, defines, strict, sphere_res):
        self.base = base_dir
        self.defs = dict(defines)
        self.strict = strict
        self.sphere_res = sphere_res
        self.ids = {}
        self.media = []  # homogeneous media in declaration order: (sigma_t, albedo rgb, g); built in finish()
        self.out = XMLScene()
        self.sc = scenes.Scene()
        self.mat_index = {}  # id(pg_material) -> scene material index

    # -- helpers
    def attr(self, el, name, default=None):
        v = el.get(name, default)
        if isinstance(v, str) and "$" in v:
            v = re.sub(r"\$(\w+)", lambda m: str(self.defs[m.group(1)]), v)
        return v

    def unsupported(self, tag, typ, reason):
        if self.strict:
            raise NotImplementedError(f"<{tag} type=\"{typ}\">: {reason}")
        self.out.skipped.append((tag, typ, reason))

    def props(self, el):
        """Properties of an element: name -> python value (floats, ints, bools, strings, rgb arrays,
        4x4 matrices for transforms)."""
        P = {}
        for c in el:
            name = self.attr(c, "name")
            tag = c.tag
            if tag in ("float",):
                P[name] = float(self.attr(c, "value"))
            elif tag == "integer":
                P[name] = int(self.attr(c, "value"))
            elif tag == "boolean":
                P[name] = self.attr(c, "value").strip().lower() == "true"
            elif tag == "string":
                P[name] = self.attr(c, "value")
            elif tag in ("rgb", "srgb", "spectrum", "color"):
                v = self.attr(c, "value")
                if ":" in v:
                    raise NotImplementedError(f"<{tag} name=\"{name}\">: sampled spectra need Mitsuba's spectral "
                                              "to RGB conversion; give an rgb value")
                f = _floats(v)
                rgb = np.array(f * 3 if len(f) == 1 else f[:3], np.float64)
                P[name] = _srgb_to_linear(rgb) if tag == "srgb" else rgb
            elif tag in ("point", "vector"):
                P[name] = np.array([float(self.attr(c, k, "0")) for k in "xyz"])
            elif tag == "transform":
                P[name] = self.transform(c)
        return P

    def transform(self, el):
        M = np.eye(4)
        for op in el:
            if op.tag == "translate":
                T = np.eye(4)
                T[:3, 3] = [float(self.attr(op, k, "0")) for k in "xyz"]
            elif op.tag == "rotate":
                T = _rotate([float(self.attr(op, k, "0")) for k in "xyz"], float(self.attr(op, "angle")))
            elif op.tag == "scale":
                if op.get("value") is not None:
                    v = float(self.attr(op, "value"))
                    sv = [v, v, v]
                else:
                    sv = [float(self.attr(op, k, "1")) for k in "xyz"]
                T = np.diag(sv + [1.0])
            elif op.tag == "matrix":
                T = np.array(_floats(self.attr(op, "value")), np.float64).reshape(4, 4)
            elif op.tag == "lookat":
                T = _lookat(_floats(self.attr(op, "origin")), _floats(self.attr(op, "target")),
                            _floats(self.attr(op, "up", "0, 1, 0")))
            else:
                raise NotImplementedError(f"transform operation <{op.tag}>")
            M = T @ M
        return M

    def path(self, p):
        return p if os.path.isabs(p) else os.path.join(self.base, p)

    # -- BSDFs (src/bsdfs/*.cpp constructors)
    def bsdf(self, el):
        typ = self.attr(el, "type")
        P = self.props(el)
        nested = [c for c in el if c.tag == "bsdf" or c.tag == "ref"]
        for c in el:
            if c.tag == "texture":
                raise NotImplementedError(f"<bsdf type=\"{typ}\">: textures are out of scope (constant albedos only)")

        def ior(name, default):
            v = P.get(name, default)
            return float(v) if not isinstance(v, str) else IOR[v.lower()]

        def rough():
            dist = P.get("distribution", "beckmann").lower()
            if dist not in ("beckmann", "ggx"):
                raise NotImplementedError(f"microfacet distribution '{dist}' (beckmann and ggx are supported)")
            a = P.get("alpha", 0.1)
            return dict(distribution=dist, alpha_u=P.get("alphaU", a), alpha_v=P.get("alphaV", a),
                        sample_visible=P.get("sampleVisible", True))

        def rgb(name, default):
            a = np.asarray(P.get(name, default), np.float64).reshape(-1)
            return tuple((a if a.size == 3 else np.repeat(a[:1], 3)).tolist())

        if typ == "twosided":
            if not nested:
                raise ValueError("twosided needs a nested bsdf")
            m = self.child_bsdf(nested[0])
            m2 = capi.pg_material.from_buffer_copy(m)
            m2.flags |= capi.PG_MAT_TWOSIDED
            return m2
        if typ == "diffuse":
            return scenes.material("diffuse", reflectance=rgb("reflectance", 0.5))
        if typ in ("conductor", "roughconductor"):
            kw = rough() if typ == "roughconductor" else {}
            name = P.get("material", "Cu")
            if "eta" in P or "k" in P:
                kw.update(eta=rgb("eta", 0.0), k=rgb("k", 1.0), conductor="none")
            elif name.lower() == "none":
                kw.update(conductor="none")
            elif name in scenes.CONDUCTORS:
                kw.update(conductor=name)
            else:
                raise ValueError(f"conductor material '{name}' is not one of the reference's data/ior presets")
            m = scenes.material(typ, specular_reflectance=rgb("specularReflectance", 1.0), **kw)
            if "extEta" in P:  # roughconductor.cpp:173-188: eta and k are relative to the exterior
                ext = ior("extEta", "air")
                m.eta = scenes._f4([x / ext for x in m.eta[:3]])
                m.k = scenes._f4([x / ext for x in m.k[:3]])
            return m
        if typ in ("dielectric", "roughdielectric"):
            kw = rough() if typ == "roughdielectric" else {}
            return scenes.material(typ, int_ior=ior("intIOR", "bk7"), ext_ior=ior("extIOR", "air"),
                                   specular_reflectance=rgb("specularReflectance", 1.0),
                                   specular_transmittance=rgb("specularTransmittance", 1.0), **kw)
        if typ in ("plastic", "roughplastic"):
            kw = rough() if typ == "roughplastic" else {}
            if typ == "roughplastic" and kw["alpha_u"] != kw["alpha_v"]:
                raise NotImplementedError("roughplastic is isotropic")
            kw.pop("alpha_v", None)
            if typ == "roughplastic":
                kw["alpha"] = kw.pop("alpha_u")
            return scenes.material(typ, int_ior=ior("intIOR", "polypropylene"), ext_ior=ior("extIOR", "air"),
                                   diffuse_reflectance=rgb("diffuseReflectance", 0.5),
                                   specular_reflectance=rgb("specularReflectance", 1.0),
                                   nonlinear=P.get("nonlinear", False), **kw)
        if typ == "null":
            return scenes.material("null")
        raise NotImplementedError(f"<bsdf type=\"{typ}\"> is not on the GPU path's BSDF set")

    def child_bsdf(self, el, top=False):
        if el.tag == "ref":
            obj = self.ids[self.attr(el, "id")]
            if not isinstance(obj, capi.pg_material):
                raise ValueError(f"<ref id=\"{el.get('id')}\"> is not a bsdf")
            return obj
        m = self.bsdf(el)
        if top:
            self.out.bsdfs.append((el.get("id") or self.attr(el, "type"), m))
        if el.get("id"):
            self.ids[el.get("id")] = m
        return m

    def material_index(self, m):
        k = id(m)
        if k not in self.mat_index:
            self.mat_index[k] = self.sc.add_material(m)
        return self.mat_index[k]

    # -- meshes
    def mesh(self, el, typ, P):
        if typ == "obj":
            V, F, N = _read_obj(self.path(P["filename"]))
        elif typ == "ply":
            V, F, N = _read_ply(self.path(P["filename"]))
        elif typ == "rectangle":  # src/shapes/rectangle.cpp: [-1, 1]^2 at z = 0, normal +z
            V = np.array([[-1, -1, 0], [1, -1, 0], [1, 1, 0], [-1, 1, 0]], np.float64)
            F = np.array([[0, 1, 2], [2, 3, 0]])
            N = np.tile([0.0, 0.0, 1.0], (4, 1))
        elif typ == "cube":  # src/shapes/cube.cpp: [-1, 1]^3, 24 vertices, outward normals
            Vs, Fs, Ns = [], [], []
            for axis in range(3):
                for sgn in (-1.0, 1.0):
                    n = np.zeros(3)
                    n[axis] = sgn
                    u, v = np.zeros(3), np.zeros(3)
                    u[(axis + 1) % 3], v[(axis + 2) % 3] = 1, 1
                    c = n
                    quad = [c - u - v, c + u - v, c + u + v, c - u + v]
                    b = 4 * len(Vs)
                    f = [[b, b + 1, b + 2], [b + 2, b + 3, b]]
                    if np.dot(np.cross(quad[1] - quad[0], quad[2] - quad[0]), n) < 0:
                        f = [[x[0], x[2], x[1]] for x in f]
                    Vs.append(quad)
                    Fs += f
                    Ns.append([n] * 4)
            V, F, N = np.concatenate(Vs), np.array(Fs), np.concatenate(Ns)
        elif typ == "disk":  # analytic in the reference (src/shapes/disk.cpp): unit disk, normal +z
            n = 4 * self.sphere_res[0]
            ang = np.arange(n) * 2 * np.pi / n
            V = np.concatenate([[[0, 0, 0]], np.stack([np.cos(ang), np.sin(ang), np.zeros(n)], 1)])
            F = np.array([[0, 1 + i, 1 + (i + 1) % n] for i in range(n)])
            N = np.tile([0.0, 0.0, 1.0], (n + 1, 1))
        elif typ == "sphere":  # analytic in the reference (src/shapes/sphere.cpp): tessellated here
            c = P.get("center", np.zeros(3))
            r = float(P.get("radius", 1.0))
            V, F, N = scenes.uv_sphere(c, r, *self.sphere_res)
            V, N = V.astype(np.float64), N.astype(np.float64)
        elif typ == "serialized":  # src/shapes/serialized.cpp:148-210
            if "maxSmoothAngle" in P:
                self.unsupported("shape", typ, "maxSmoothAngle (TriMesh::rebuildTopology) is not restated; "
                                 "the file's normals or smooth vertex normals are used")
            V, F, N = read_serialized(self.path(P["filename"]), int(P.get("shapeIndex", 0)))
        else:
            return None
        V, F = np.asarray(V, np.float64), np.asarray(F, np.int64)
        M = P.get("toWorld", np.eye(4))
        V = V @ M[:3, :3].T + M[:3, 3]
        face = P.get("faceNormals", False)
        if N is not None and not face:
            Nt = np.asarray(N, np.float64) @ np.linalg.inv(M[:3, :3])  # normals: inverse transpose
            N = Nt / np.maximum(np.linalg.norm(Nt, axis=1, keepdims=True), 1e-30)
        elif not face:
            N = _vertex_normals(V, F)
        flip = P.get("flipNormals", False)
        if np.linalg.det(M[:3, :3]) < 0 and typ in ("rectangle", "cube", "disk", "sphere"):
            F = F[:, ::-1]
        elif np.linalg.det(M[:3, :3]) < 0 and typ == "serialized":
            F = F[:, [1, 0, 2]]  # serialized.cpp:197-202 swaps idx[0] and idx[1]
        if face:
            if flip:
                F = F[:, ::-1]
            return V, F, None
        if flip:
            N = -N
        return V, F, N

    def shape(self, el):
        typ = self.attr(el, "type")
        P = self.props(el)
        if typ in ("shapegroup", "instance", "hair", "heightfield", "cylinder"):
            return self.unsupported("shape", typ, "not flattened by this loader")
        res = self.mesh(el, typ, P)
        if res is None:
            return self.unsupported("shape", typ, "unknown shape plugin")
        V, F, N = res
        mat = None
        radiance = None
        sides = {"interior": -1, "exterior": -1}
        for c in el:
            if c.tag in ("bsdf", "ref") and (c.tag == "bsdf" or isinstance(self.ids.get(c.get("id")), capi.pg_material)):
                mat = self.child_bsdf(c)
            elif c.tag == "emitter":
                et = self.attr(c, "type")
                if et != "area":
                    raise NotImplementedError(f"<emitter type=\"{et}\"> inside a shape")
                ep = self.props(c)
                radiance = tuple(np.asarray(ep.get("radiance", np.ones(3))).reshape(-1).tolist())
                if len(radiance) == 1:
                    radiance = radiance * 3
            elif c.tag == "medium" or (c.tag == "ref" and c.get("name") in ("interior", "exterior")):
                side = self.attr(c, "name")
                if side not in sides:
                    raise ValueError(f"<{c.tag}> in a shape needs name=\"interior\" or \"exterior\"")
                if c.tag == "medium":
                    sides[side] = self.medium(c)
                else:
                    obj = self.ids.get(self.attr(c, "id"))
                    if not (isinstance(obj, tuple) and obj[0] == "medium"):
                        raise ValueError(f"<ref id=\"{c.get('id')}\"> is not a medium")
                    sides[side] = obj[1]
        transition = sides["interior"] >= 0 or sides["exterior"] >= 0
        if mat is None:  # Shape::configure (shape.cpp:48-72)
            if radiance is not None:
                mat = scenes.material("diffuse", reflectance=(0.0, 0.0, 0.0))
            elif transition:
                mat = scenes.material("null")
            else:
                mat = scenes.material("diffuse", reflectance=(0.5, 0.5, 0.5))
        m = self.material_index(mat)
        self.sc.add_mesh(V.astype(np.float32), F.astype(np.uint32), None if N is None else N.astype(np.float32),
                         material=m, radiance=radiance, interior=sides["interior"], exterior=sides["exterior"])

    # -- participating media (src/medium/homogeneous.cpp, materials.h:90-195 lookupMaterial)
    def medium(self, el):
        typ = self.attr(el, "type")
        if typ != "homogeneous":
            raise NotImplementedError(f"<medium type=\"{typ}\">: only homogeneous media are flattened from XML "
                                      "(heterogeneous grids are built with Scene.add_medium)")
        P = self.props(el)
        if "material" in P:
            raise NotImplementedError("<medium>: material presets (materials.h) are not restated; give sigmaS/sigmaA "
                                      "or sigmaT/albedo")
        has_as, has_ta = "sigmaS" in P or "sigmaA" in P, "sigmaT" in P or "albedo" in P
        if has_as and has_ta:
            raise ValueError("<medium>: sigmaS & sigmaA *or* sigmaT & albedo (materials.h:104-106)")
        one = np.ones(3)
        if has_ta:
            st, alb = np.asarray(P.get("sigmaT", one), np.float64), np.asarray(P.get("albedo", one), np.float64)
            ss, sa = alb * st, st - alb * st
        else:  # the Skin1 default preset is not restated: both coefficients must then be given
            if not has_as:
                raise NotImplementedError("<medium>: no coefficients (the default Skin1 preset is not restated)")
            ss, sa = np.asarray(P.get("sigmaS", 0 * one), np.float64), np.asarray(P.get("sigmaA", 0 * one), np.float64)
        g_red = float(P.get("g", 0.0)) if not isinstance(P.get("g", 0.0), np.ndarray) else float(P["g"][0])
        scale = float(P.get("scale", 1.0))
        ss, sa = ss * (1 - g_red) * scale, sa * scale  # Medium::Medium reduced scattering, then lookupMaterial scale
        st = ss + sa
        if not np.allclose(st, st[0], rtol=1e-6):
            raise NotImplementedError("<medium>: chromatic sigmaT (the GPU medium has one extinction per point)")
        if not st[0] > 0:
            raise ValueError("<medium>: sigmaT must be > 0")
        g = 0.0
        for c in el:
            if c.tag == "phase":
                pt = self.attr(c, "type")
                if pt == "hg":
                    g = float(self.props(c).get("g", 0.8))  # hg.cpp:50
                elif pt != "isotropic":
                    raise NotImplementedError(f"<phase type=\"{pt}\"> (hg and isotropic only)")
        self.media.append((float(st[0]), tuple((ss / st).tolist()), g))
        idx = len(self.media) - 1
        if el.get("id"):
            self.ids[el.get("id")] = ("medium", idx)
        return idx

    def finish_media(self):
        """A homogeneous medium is a constant density over a box that holds the whole scene (shape
        bounds enlarged by their extent): paths only enter it through transition surfaces and end at
        scene geometry, so the box bounds nothing that matters."""
        if not self.media:
            return
        P = np.concatenate(self.sc._pos)
        lo, hi = P.min(0), P.max(0)
        ext = float((hi - lo).max()) + 1e-3
        for st, alb, g in self.media:
            self.sc.add_medium(np.ones((2, 2, 2), np.float32), tuple((lo - ext).tolist()), tuple((hi + ext).tolist()),
                               st, alb, g)

    # -- emitters, sensor, integrator
    def emitter(self, el):
        typ = self.attr(el, "type")
        P = self.props(el)
        R = P.get("toWorld", np.eye(4))[:3, :3]
        if typ == "envmap":
            try:
                rgb = read_image(self.path(P["filename"]))
            except (NotImplementedError, OSError) as e:
                return self.unsupported("emitter", typ, f"{P['filename']}: {e}")
            self.sc.set_envmap(rgb, to_world=R, scale=float(P.get("scale", 1.0)))
        elif typ == "constant":  # src/emitters/constant.cpp: uniform radiance, sampled through the envmap CDFs
            rad = np.asarray(P.get("radiance", np.ones(3)), np.float32).reshape(-1)
            self.sc.set_envmap(np.ones((16, 32, 3), np.float32) * (rad if rad.size == 3 else rad[0]), to_world=R)
        else:
            self.unsupported("emitter", typ, "only area (in a shape), envmap and constant emitters")

    def sensor(self, el):
        typ = self.attr(el, "type")
        if typ != "perspective":
            raise NotImplementedError(f"<sensor type=\"{typ}\"> (perspective only)")
        P = self.props(el)
        W, H = 768, 576  # hdrfilm defaults (src/films/hdrfilm.cpp)
        for c in el:
            if c.tag == "film":
                fp = self.props(c)
                W, H = int(fp.get("width", W)), int(fp.get("height", H))
            elif c.tag == "sampler":
                sp = self.props(c)
                self.out.spp = int(sp.get("sampleCount", 4))
        fov = float(P.get("fov", 30.0)) if "fov" in P else None
        if fov is None and "focalLength" in P:
            f = float(str(P["focalLength"]).replace("mm", ""))
            fov = math.degrees(2 * math.atan(36.0 / (2 * f)))  # 35 mm film, fovAxis x (perspective.cpp)
        fov = 39.3077 if fov is None else fov
        axis = P.get("fovAxis", "x").lower()
        t = math.tan(math.radians(fov) / 2)
        if axis == "y" or (axis == "smaller" and H < W) or (axis == "larger" and H > W):
            t = t * W / H
        elif axis == "diagonal":
            t = t * W / math.hypot(W, H)
        fov_x = math.degrees(2 * math.atan(t))
        M = P.get("toWorld", np.eye(4))
        o = M[:3, 3]
        d = M[:3, :3] @ [0, 0, 1]
        up = M[:3, :3] @ [0, 1, 0]
        left_m = M[:3, :3] @ [1, 0, 0]
        left = np.cross(up, d)
        self.sc.mirror_x = bool(np.dot(left, left_m) < 0)
        self.sc.set_camera(tuple(o), tuple(o + d / np.linalg.norm(d)), tuple(up / np.linalg.norm(up)), fov_x, W, H,
                           near=float(P.get("nearClip", 1e-2)), far=float(P.get("farClip", 1e4)))

    def run(self, root):
        if root.tag != "scene":
            raise ValueError("not a Mitsuba scene file")
        for el in root:
            if el.tag == "default":
                self.defs.setdefault(el.get("name"), el.get("value"))
        for el in root:
            if el.tag == "integrator":
                self.out.integrator_type = self.attr(el, "type")
                self.out.integrator_props = {k: (v.tolist() if isinstance(v, np.ndarray) else v)
                                             for k, v in self.props(el).items()}
            elif el.tag == "sensor":
                self.sensor(el)
            elif el.tag == "bsdf":
                try:
                    self.child_bsdf(el, top=True)
                except NotImplementedError as e:
                    if self.strict:
                        raise
                    self.out.skipped.append(("bsdf", self.attr(el, "type"), str(e)))
            elif el.tag == "shape":
                self.shape(el)
            elif el.tag == "emitter":
                self.emitter(el)
            elif el.tag in ("default", "include"):
                if el.tag == "include":
                    self.run(ET.parse(self.path(self.attr(el, "filename"))).getroot())
            elif el.tag == "medium":
                try:
                    self.medium(el)
                except NotImplementedError as e:
                    if self.strict:
                        raise
                    self.out.skipped.append(("medium", self.attr(el, "type"), str(e)))
            elif el.tag in ("phase", "texture"):
                self.unsupported(el.tag, self.attr(el, "type"), "not flattened by this loader")
        return self.out


def load(source, defines=None, strict=True, sphere_res=(64, 32)):
    """Parse a Mitsuba 0.5 scene (a path, or the XML text itself) into an XMLScene.  `defines` are the
    -D key=value substitutions (mitsuba.cpp:154).  The Scene is finalized when it has shapes and a
    camera (BSDF-only files such as data/tests/test_bsdf.xml return scene = None)."""
    if os.path.exists(str(source)):
        root = ET.parse(source).getroot()
        base = os.path.dirname(os.path.abspath(source))
    else:
        root = ET.fromstring(source)
        base = os.getcwd()
    L = _Loader(base, defines or {}, strict, sphere_res)
    out = L.run(root)
    L.finish_media()
    if L.sc.shapes and L.sc.camera is not None:
        out.scene = L.sc.finalize()
    elif L.sc.shapes:
        out.scene = L.sc
    return out


# ---- mesh and image readers ----------------------------------------------------------------------
def _vertex_normals(V, F):
    """TriMesh::computeNormals (trimesh.cpp:636-680): face normals weighted by the corner angle."""
    N = np.zeros_like(V)
    tri = V[F]
    fn = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    ln = np.linalg.norm(fn, axis=1, keepdims=True)
    ok = ln[:, 0] > 0
    fn = fn / np.maximum(ln, 1e-300)
    for i in range(3):
        a = tri[:, (i + 1) % 3] - tri[:, i]
        b = tri[:, (i + 2) % 3] - tri[:, i]
        a /= np.maximum(np.linalg.norm(a, axis=1, keepdims=True), 1e-300)
        b /= np.maximum(np.linalg.norm(b, axis=1, keepdims=True), 1e-300)
        ang = 2 * np.arcsin(np.clip(np.linalg.norm(a - b, axis=1) / 2, 0, 1))  # unitAngle
        np.add.at(N, F[ok, i], fn[ok] * ang[ok, None])
    ln = np.linalg.norm(N, axis=1, keepdims=True)
    return np.where(ln > 0, N / np.maximum(ln, 1e-300), np.array([1.0, 0.0, 0.0]))


def _read_obj(path):
    """Wavefront OBJ (src/shapes/obj.cpp): v / vn / f (polygons fanned); vertices are welded by
    their (position, normal) index pair."""
    P, Nn, keys, faces = [], [], {}, []
    has_n = False
    with open(path) as f:
        for line in f:
            t = line.split()
            if not t or t[0].startswith("#"):
                continue
            if t[0] == "v":
                P.append([float(x) for x in t[1:4]])
            elif t[0] == "vn":
                Nn.append([float(x) for x in t[1:4]])
            elif t[0] == "f":
                idx = []
                for w in t[1:]:
                    parts = w.split("/")
                    vi = int(parts[0])
                    vi = vi - 1 if vi > 0 else len(P) + vi
                    ni = -1
                    if len(parts) >= 3 and parts[2]:
                        ni = int(parts[2])
                        ni = ni - 1 if ni > 0 else len(Nn) + ni
                        has_n = True
                    k = (vi, ni)
                    if k not in keys:
                        keys[k] = len(keys)
                    idx.append(keys[k])
                for j in range(1, len(idx) - 1):
                    faces.append([idx[0], idx[j], idx[j + 1]])
    order = sorted(keys.items(), key=lambda kv: kv[1])
    V = np.array([P[k[0]] for k, _ in order], np.float64)
    N = np.array([Nn[k[1]] if k[1] >= 0 else [0, 0, 0] for k, _ in order], np.float64) if has_n else None
    return V, np.array(faces, np.int64), N


# TriMesh serialization flags (trimesh.cpp:89-97) and file header (trimesh.cpp:34-36)
_SER_HEADER, _SER_V3, _SER_V4 = 0x041C, 0x0003, 0x0004
_SER_NORMALS, _SER_TEXCOORDS, _SER_COLORS, _SER_FACE_NORMALS = 0x0001, 0x0002, 0x0008, 0x0010
_SER_SINGLE, _SER_DOUBLE = 0x1000, 0x2000


def read_serialized(path, index=0):
    """Mesh `index` of a Mitsuba .serialized file (TriMesh::loadCompressed / readHeader / readOffset,
    trimesh.cpp:175-294): a little-endian (u16 0x041C, u16 version) header, then a zlib stream of
    u32 flags, [v4: NUL-terminated name], u64 vertex and triangle counts, positions, [normals],
    [texcoords], [colors] (f32 or f64 by flag) and u32 triangle indices.  Files with several meshes
    end with a dictionary of per-mesh byte offsets (u64 in v4, u32 in v3) and a u32 mesh count.
    Returns (V, F, N or None) as float64 / int64 arrays."""
    with open(path, "rb") as f:
        data = f.read()

    def header(off):
        fmt, ver = struct.unpack_from("<HH", data, off)
        if fmt == 0x1C04:
            raise ValueError(f"{path}: geometry file of an old Mitsuba version (re-import it)")
        if fmt != _SER_HEADER or ver not in (_SER_V3, _SER_V4):
            raise ValueError(f"{path}: not a serialized mesh (header {fmt:#06x}, version {ver})")
        return ver

    version = header(0)
    off = 0
    if index != 0:
        count = struct.unpack_from("<I", data, len(data) - 4)[0]
        if index < 0 or index >= count:
            raise ValueError(f"{path}: shape index {index} out of range 0..{count - 1}")
        if version == _SER_V4:
            off = struct.unpack_from("<Q", data, len(data) - 8 * (count - index) - 4)[0]
        else:
            off = struct.unpack_from("<I", data, len(data) - 4 * (count - index + 1))[0]
        version = header(off)
    z = zlib.decompressobj()
    raw = z.decompress(data[off + 4:])
    pos = 0
    flags = struct.unpack_from("<I", raw, pos)[0]
    pos += 4
    if version == _SER_V4:
        pos = raw.index(b"\0", pos) + 1
    nv, nt = struct.unpack_from("<QQ", raw, pos)
    pos += 16
    ft = np.dtype("<f8") if flags & _SER_DOUBLE else np.dtype("<f4")

    def take(dt, n):
        nonlocal pos
        a = np.frombuffer(raw, dt, n, pos)
        pos += dt.itemsize * n
        return a

    V = take(ft, 3 * nv).reshape(nv, 3).astype(np.float64)
    N = take(ft, 3 * nv).reshape(nv, 3).astype(np.float64) if flags & _SER_NORMALS else None
    if flags & _SER_TEXCOORDS:
        take(ft, 2 * nv)
    if flags & _SER_COLORS:
        take(ft, 3 * nv)
    F = take(np.dtype("<u4"), 3 * nt).reshape(nt, 3).astype(np.int64)
    if nv and (F.min() < 0 or F.max() >= nv):
        raise ValueError(f"{path}: triangle index out of range")
    return V, F, N


def write_serialized(path, meshes):
    """Write meshes [(V, F, N or None[, name])] as a version-4 .serialized file, float32, the layout of
    TriMesh::serialize (trimesh.cpp:1131-1176) plus the offset dictionary of a multi-mesh file."""
    out, offsets = bytearray(), []
    for m in meshes:
        V, F, N = m[0], m[1], m[2]
        name = m[3] if len(m) > 3 else ""
        flags = _SER_SINGLE | (_SER_NORMALS if N is not None else 0)
        body = struct.pack("<I", flags) + name.encode() + b"\0" + struct.pack("<QQ", len(V), len(F))
        body += np.asarray(V, "<f4").tobytes()
        if N is not None:
            body += np.asarray(N, "<f4").tobytes()
        body += np.asarray(F, "<u4").tobytes()
        offsets.append(len(out))
        out += struct.pack("<HH", _SER_HEADER, _SER_V4) + zlib.compress(body)
    out += np.asarray(offsets, "<u8").tobytes() + struct.pack("<I", len(meshes))
    with open(path, "wb") as f:
        f.write(bytes(out))


_PLY_TYPES = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
              "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
              "float": "f4", "float32": "f4", "double": "f8", "float64": "f8"}


def _read_ply(path):
    """Stanford PLY (src/shapes/ply.cpp): ascii or binary, vertex x y z [nx ny nz], face vertex lists."""
    with open(path, "rb") as f:
        data = f.read()
    end = data.index(b"end_header") + len(b"end_header")
    while data[end:end + 1] in (b"\r", b"\n"):
        end += 1
    header = data[:end].decode("ascii").splitlines()
    fmt, elems = None, []
    for line in header:
        t = line.split()
        if not t:
            continue
        if t[0] == "format":
            fmt = t[1]
        elif t[0] == "element":
            elems.append([t[1], int(t[2]), []])
        elif t[0] == "property":
            elems[-1][2].append(t[1:])
    body = data[end:]
    V = F = N = None
    if fmt == "ascii":
        toks = body.split()
        pos = 0
        for name, count, props in elems:
            rows = []
            for _ in range(count):
                row = []
                for p in props:
                    if p[0] == "list":
                        n = int(toks[pos])
                        row.append([int(x) for x in toks[pos + 1:pos + 1 + n]])
                        pos += 1 + n
                    else:
                        row.append(float(toks[pos]))
                        pos += 1
                rows.append(row)
            V, F, N = _ply_collect(name, props, rows, V, F, N)
    else:
        endian = "<" if fmt == "binary_little_endian" else ">"
        pos = 0
        for name, count, props in elems:
            if all(p[0] != "list" for p in props):
                dt = np.dtype([(p[1], endian + _PLY_TYPES[p[0]]) for p in props])
                arr = np.frombuffer(body, dt, count, pos)
                pos += dt.itemsize * count
                rows = arr
            else:
                rows = []
                for _ in range(count):
                    row = []
                    for p in props:
                        if p[0] == "list":
                            ct, it = _PLY_TYPES[p[1]], _PLY_TYPES[p[2]]
                            n = int(np.frombuffer(body, endian + ct, 1, pos)[0])
                            pos += np.dtype(ct).itemsize
                            row.append(np.frombuffer(body, endian + it, n, pos).astype(np.int64).tolist())
                            pos += np.dtype(it).itemsize * n
                        else:
                            t = _PLY_TYPES[p[0]]
                            row.append(float(np.frombuffer(body, endian + t, 1, pos)[0]))
                            pos += np.dtype(t).itemsize
                    rows.append(row)
            V, F, N = _ply_collect(name, props, rows, V, F, N)
    return V, F, N


def _ply_collect(name, props, rows, V, F, N):
    names = [p[-1] for p in props]
    if name == "vertex":
        if isinstance(rows, np.ndarray):
            V = np.stack([rows[k].astype(np.float64) for k in "xyz"], 1)
            if "nx" in names:
                N = np.stack([rows[k].astype(np.float64) for k in ("nx", "ny", "nz")], 1)
        else:
            a = np.array(rows, np.float64)
            V = a[:, [names.index(k) for k in "xyz"]]
            if "nx" in names:
                N = a[:, [names.index(k) for k in ("nx", "ny", "nz")]]
    elif name == "face":
        li = [i for i, p in enumerate(props) if p[0] == "list"][0]
        tris = []
        for r in rows:
            idx = r[li]
            for j in range(1, len(idx) - 1):
                tris.append([idx[0], idx[j], idx[j + 1]])
        F = np.array(tris, np.int64)
    return V, F, N


def read_image(path):
    """Latitude-longitude RGB image for envmap: .npy (H, W, 3), .pfm, or OpenEXR scanline files with
    NONE / ZIPS / ZIP compression and half or float channels.  (PIZ and the lossy codecs need
    OpenEXR, which is not available.)"""
    ext = os.path.splitext(path)[1].lower()
    if ext == ".npy":
        return np.ascontiguousarray(np.load(path, allow_pickle=False), np.float32)[..., :3]
    if ext == ".pfm":
        with open(path, "rb") as f:
            kind = f.readline().strip()
            w, h = (int(x) for x in f.readline().split())
            scale = float(f.readline())
            a = np.frombuffer(f.read(), "<f4" if scale < 0 else ">f4")
        a = a.reshape(h, w, 3 if kind == b"PF" else 1)[::-1]
        return np.ascontiguousarray(np.repeat(a, 3, 2) if a.shape[2] == 1 else a, np.float32)
    if ext == ".exr":
        return _read_exr(path)
    raise NotImplementedError(f"image format {ext}")


def _read_exr(path):
    with open(path, "rb") as f:
        d = f.read()
    if struct.unpack_from("<I", d, 0)[0] != 20000630:
        raise ValueError("not an OpenEXR file")
    pos = 8
    attrs = {}
    while d[pos] != 0:
        name_end = d.index(b"\0", pos)
        name = d[pos:name_end].decode()
        type_end = d.index(b"\0", name_end + 1)
        size = struct.unpack_from("<i", d, type_end + 1)[0]
        attrs[name] = d[type_end + 5:type_end + 5 + size]
        pos = type_end + 5 + size
    pos += 1
    comp = attrs["compression"][0]
    if comp not in (0, 2, 3):
        raise NotImplementedError(f"OpenEXR compression {comp} (NONE, ZIPS and ZIP are supported; PIZ etc. "
                                  "need the OpenEXR library)")
    x0, y0, x1, y1 = struct.unpack_from("<iiii", attrs["dataWindow"])
    W, H = x1 - x0 + 1, y1 - y0 + 1
    ch, p = [], 0
    cl = attrs["channels"]
    while cl[p] != 0:
        e = cl.index(b"\0", p)
        cname = cl[p:e].decode()
        ptype = struct.unpack_from("<i", cl, e + 1)[0]
        ch.append((cname, ptype))
        p = e + 17
    ch.sort(key=lambda c: c[0])  # channels are stored in alphabetical order
    lines = {0: 1, 2: 1, 3: 16}[comp]
    nblocks = (H + lines - 1) // lines
    offsets = struct.unpack_from(f"<{nblocks}Q", d, pos)
    img = {c: np.zeros((H, W), np.float32) for c, _ in ch}
    for off in offsets:
        yb, size = struct.unpack_from("<ii", d, off)
        raw = d[off + 8:off + 8 + size]
        nl = min(lines, y1 - yb + 1)
        expect = sum(W * nl * (2 if t == 1 else 4) for _, t in ch)
        if comp != 0 and size < expect:
            u = np.frombuffer(zlib.decompress(raw), np.uint8).astype(np.int32)
            u = np.cumsum(np.concatenate([u[:1], u[1:] - 128])) & 0xFF  # undo the predictor
            half = (len(u) + 1) // 2
            out = np.empty(len(u), np.uint8)
            out[0::2], out[1::2] = u[:half], u[half:]  # de-interleave
            raw = out.tobytes()
        q = 0
        for yy in range(nl):
            for c, t in ch:
                dt = "<f2" if t == 1 else ("<f4" if t == 2 else "<u4")
                n = W * (2 if t == 1 else 4)
                img[c][yb - y0 + yy] = np.frombuffer(raw, dt, W, q).astype(np.float32)
                q += n
    names = [c for c, _ in ch]
    pick = [n for n in ("R", "G", "B") if n in names] or names[:3]
    rgb = np.stack([img[n] for n in pick], -1)
    return np.ascontiguousarray(np.repeat(rgb, 3, -1) if rgb.shape[-1] == 1 else rgb, np.float32)


# ---- export (the reverse direction: run a synthetic scene through the reference renderer) ----------
_KIND = {capi.PG_BSDF_DIFFUSE: "diffuse", capi.PG_BSDF_CONDUCTOR: "conductor",
         capi.PG_BSDF_ROUGHCONDUCTOR: "roughconductor", capi.PG_BSDF_DIELECTRIC: "dielectric",
         capi.PG_BSDF_ROUGHDIELECTRIC: "roughdielectric", capi.PG_BSDF_PLASTIC: "plastic",
         capi.PG_BSDF_ROUGHPLASTIC: "roughplastic", capi.PG_BSDF_NULL: "null"}


def _rgb_el(name, v):
    return f'<rgb name="{name}" value="{v[0]!r}, {v[1]!r}, {v[2]!r}"/>'


def _bsdf_xml(m):
    kind = _KIND[m.type]
    body = []
    f32 = lambda x: float(np.float32(x))
    if kind == "diffuse":
        body.append(_rgb_el("reflectance", [f32(x) for x in m.diffuse_reflectance[:3]]))
    if kind in ("conductor", "roughconductor"):
        body.append(_rgb_el("eta", [f32(x) for x in m.eta[:3]]))
        body.append(_rgb_el("k", [f32(x) for x in m.k[:3]]))
        body.append(_rgb_el("specularReflectance", [f32(x) for x in m.specular_reflectance[:3]]))
        body.append('<float name="extEta" value="1"/>')
    if kind in ("dielectric", "roughdielectric", "plastic", "roughplastic"):
        body.append(f'<float name="intIOR" value="{f32(m.int_ior)!r}"/>')
        body.append(f'<float name="extIOR" value="{f32(m.ext_ior)!r}"/>')
    if kind in ("dielectric", "roughdielectric"):
        body.append(_rgb_el("specularReflectance", [f32(x) for x in m.specular_reflectance[:3]]))
        body.append(_rgb_el("specularTransmittance", [f32(x) for x in m.specular_transmittance[:3]]))
    if kind in ("plastic", "roughplastic"):
        body.append(_rgb_el("diffuseReflectance", [f32(x) for x in m.diffuse_reflectance[:3]]))
        body.append(_rgb_el("specularReflectance", [f32(x) for x in m.specular_reflectance[:3]]))
        body.append(f'<boolean name="nonlinear" value="{"true" if m.flags & capi.PG_MAT_NONLINEAR else "false"}"/>')
    if kind.startswith("rough"):
        body.append(f'<string name="distribution" value="{"ggx" if m.distribution == capi.PG_DIST_GGX else "beckmann"}"/>')
        if kind == "roughplastic":
            body.append(f'<float name="alpha" value="{f32(m.alpha_u)!r}"/>')
        else:
            body.append(f'<float name="alphaU" value="{f32(m.alpha_u)!r}"/>')
            body.append(f'<float name="alphaV" value="{f32(m.alpha_v)!r}"/>')
        body.append(f'<boolean name="sampleVisible" value="{"false" if m.flags & capi.PG_MAT_SAMPLE_ALL else "true"}"/>')
    inner = f'<bsdf type="{kind}">' + "".join(body) + "</bsdf>"
    if m.flags & capi.PG_MAT_TWOSIDED:
        inner = f'<bsdf type="twosided">{inner}</bsdf>'
    return inner


def save(scene, path, spp=64, integrator="path"):
    """Write `scene` as a Mitsuba 0.5 scene: one OBJ per shape (positions, normals), inline BSDFs,
    area emitters, the perspective sensor (lookat + fov along x), a box-filtered hdrfilm, and the
    environment map as a PFM.  load(path) reads it back to the same arrays."""
    d = os.path.dirname(os.path.abspath(path))
    stem = os.path.splitext(os.path.basename(path))[0]
    os.makedirs(d, exist_ok=True)
    sc = scene.desc() and scene
    P, N, I = sc.positions, sc.normals, sc.indices
    out = ['<?xml version="1.0" encoding="utf-8"?>', '<scene version="0.5.0">',
           f'<integrator type="{integrator}"/>']
    cam = sc.camera
    v3 = lambda a: f"{a[0]!r}, {a[1]!r}, {a[2]!r}"
    f32l = lambda a: [float(np.float32(x)) for x in a]
    out.append(f'<sensor type="perspective"><float name="fov" value="{float(np.float32(cam.fov_x_deg))!r}"/>'
               f'<string name="fovAxis" value="x"/><float name="nearClip" value="{float(np.float32(cam.near_clip))!r}"/>'
               f'<float name="farClip" value="{float(np.float32(cam.far_clip))!r}"/>'
               f'<transform name="toWorld"><lookat origin="{v3(f32l(cam.origin))}" target="{v3(f32l(cam.target))}" '
               f'up="{v3(f32l(cam.up))}"/></transform>'
               f'<sampler type="independent"><integer name="sampleCount" value="{int(spp)}"/></sampler>'
               f'<film type="hdrfilm"><integer name="width" value="{cam.width}"/><integer name="height" '
               f'value="{cam.height}"/><rfilter type="box"/></film></sensor>')
    for si, sh in enumerate(sc.shapes):
        F = I[sh.tri_begin:sh.tri_begin + sh.tri_count].astype(np.int64)
        used = np.unique(F)
        remap = np.full(int(used.max()) + 1, -1, np.int64)
        remap[used] = np.arange(len(used))
        fn = f"{stem}_shape{si}.obj"
        with open(os.path.join(d, fn), "w") as f:
            for p in P[used]:
                f.write(f"v {float(p[0])!r} {float(p[1])!r} {float(p[2])!r}\n")
            for n in N[used]:
                f.write(f"vn {float(n[0])!r} {float(n[1])!r} {float(n[2])!r}\n")
            for t in remap[F] + 1:
                f.write(f"f {t[0]}//{t[0]} {t[1]}//{t[1]} {t[2]}//{t[2]}\n")
        em = ""
        if sh.emitter >= 0:
            r = f32l(sc.emitters[sh.emitter].radiance[:3])
            em = f'<emitter type="area">{_rgb_el("radiance", r)}</emitter>'
        out.append(f'<shape type="obj"><string name="filename" value="{fn}"/>'
                   f'{_bsdf_xml(sc.materials[sh.material])}{em}</shape>')
    if sc.envmap is not None:
        fn = f"{stem}_envmap.pfm"
        img = np.ascontiguousarray(sc._env_rgb[::-1], "<f4")
        with open(os.path.join(d, fn), "wb") as f:
            f.write(b"PF\n%d %d\n-1.0\n" % (img.shape[1], img.shape[0]))
            f.write(img.tobytes())
        R = np.asarray(list(sc.envmap.to_world), np.float64).reshape(3, 3)
        M = np.eye(4)
        M[:3, :3] = R
        out.append(f'<emitter type="envmap"><string name="filename" value="{fn}"/>'
                   f'<float name="scale" value="{float(np.float32(sc.envmap.scale))!r}"/>'
                   f'<transform name="toWorld"><matrix value="{" ".join(repr(float(x)) for x in M.reshape(-1))}"/>'
                   f'</transform></emitter>')
    out.append("</scene>")
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")
    return path
