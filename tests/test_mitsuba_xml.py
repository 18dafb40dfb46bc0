"""Mitsuba XML scene subset (mitsuba_xml.py), on the CPU.

* The reference's own BSDF test scene, data/tests/test_bsdf.xml (kept as tests/golden/test_bsdf.xml),
  loads into exactly the materials the oracle's chi-square tests use for the supported entries; the
  unsupported plugins are reported, not silently dropped.
* data/tests/test_emitter.xml: the shape loads, the PIZ envmap is reported as unreadable here.
* Export -> load round trip of synthetic scenes (OBJ meshes, BSDFs, area lights, camera, envmap as
  PFM) reproduces the triangles, materials and camera, and renders the same image in the oracle.
* Transforms, named IORs, analytic shapes, fovAxis and $-defines follow the reference's semantics.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN


def test_test_bsdf_xml_subset(pg, O):
    X = pg.mitsuba_xml
    out = X.load(os.path.join(GOLDEN, "test_bsdf.xml"), strict=False)
    names = [n for n, _ in out.bsdfs]
    assert names == ["plastic", "plastic", "diffuse", "twosided", "conductor", "dielectric", "roughdielectric",
                     "roughdielectric", "roughconductor", "roughplastic"]
    assert len(out.skipped) == 19
    skipped = {t for _, t, _ in out.skipped}
    assert {"roughdiffuse", "difftrans", "mixturebsdf", "hk", "phong", "ward", "mask", "coating",
            "roughcoating"} <= skipped
    S = pg.scenes
    expect = {
        2: S.material("diffuse", reflectance=(0.5, 0.5, 0.5)),
        3: S.material("diffuse", reflectance=(0.5, 0.5, 0.5), twosided=True),
        5: S.material("dielectric", int_ior=1.3330, ext_ior=1.000277),  # intIOR "water", extIOR "air"
        6: S.material("roughdielectric", int_ior=1.5, ext_ior=1.0, alpha=0.3),
        7: S.material("roughdielectric", int_ior=1.5, ext_ior=1.0, alpha=0.3, distribution="ggx"),
        8: S.material("roughconductor", conductor="Cu", alpha=0.3),
        9: S.material("roughplastic", alpha=0.7),
    }
    for i, m in expect.items():
        assert bytes(out.bsdfs[i][1]) == bytes(m), names[i]
    # the loaded materials behave identically in the oracle (same BSDF queries bit for bit)
    rng = np.random.default_rng(0)
    wi = rng.normal(size=(256, 3)).astype(np.float32)
    wi[:, 2] = np.abs(wi[:, 2])
    wi /= np.linalg.norm(wi, axis=1, keepdims=True)
    u = rng.random((256, 3)).astype(np.float32)
    for name, m in out.bsdfs:
        a = O.bsdf_query(pg.capi, m, wi, u)
        assert np.isfinite(a).all(), name


def test_test_emitter_xml(pg):
    out = pg.mitsuba_xml.load(os.path.join(GOLDEN, "test_emitter.xml"), strict=False)
    assert out.scene is not None and len(out.scene.shapes) == 1  # <shape type="sphere"/>
    assert [s[:2] for s in out.skipped] == [("emitter", "envmap")]
    with pytest.raises(NotImplementedError):
        pg.mitsuba_xml.load(os.path.join(GOLDEN, "test_emitter.xml"), strict=True)


def _tri_soup(sc):
    out = []
    for sh in sc.shapes:
        F = sc.indices[sh.tri_begin:sh.tri_begin + sh.tri_count]
        out.append((sc.positions[F], sc.normals[F]))
    return out


@pytest.mark.parametrize("name", ["cornell", "sky"])
def test_export_load_roundtrip(pg, O, tmp_path, name):
    S = pg.scenes
    sc = S.cornell(48, 48) if name == "cornell" else S.sky_courtyard(48, 36)
    path = pg.mitsuba_xml.save(sc, str(tmp_path / f"{name}.xml"), spp=16)
    out = pg.mitsuba_xml.load(path)
    lc = out.scene
    assert out.spp == 16 and out.integrator_type == "path"
    assert len(lc.shapes) == len(sc.shapes) and len(lc.emitters) == len(sc.emitters)
    for (p0, n0), (p1, n1) in zip(_tri_soup(sc), _tri_soup(lc)):
        assert np.array_equal(p0, p1)
        assert np.allclose(n0, n1, atol=1e-6)
    for a, b in zip(sc.shapes, lc.shapes):
        assert bytes(sc.materials[a.material]) == bytes(lc.materials[b.material])
        if a.emitter >= 0:
            assert list(sc.emitters[a.emitter].radiance) == list(lc.emitters[b.emitter].radiance)
    c0, c1 = sc.camera, lc.camera
    assert (c0.width, c0.height) == (c1.width, c1.height) and abs(c0.fov_x_deg - c1.fov_x_deg) < 1e-5
    d0 = np.subtract(c0.target, c0.origin)
    d1 = np.subtract(c1.target, c1.origin)
    assert np.allclose(c0.origin, c1.origin) and np.allclose(d0 / np.linalg.norm(d0), d1 / np.linalg.norm(d1), atol=1e-6)
    if name == "sky":
        assert np.array_equal(lc._env_rgb, sc._env_rgb)
    a = O.render(O.OracleScene(pg.capi, sc), pg.capi.default_config(), 4)[0]
    b = O.render(O.OracleScene(pg.capi, lc), pg.capi.default_config(), 4)[0]
    close = np.isclose(a, b, rtol=1e-4, atol=1e-6).all(-1)
    assert close.mean() > 0.99, close.mean()


SCENE = """<scene version="0.5.0">
  <default name="res" value="40"/>
  <integrator type="path"><integer name="maxDepth" value="$depth"/></integrator>
  <bsdf type="roughplastic" id="red"><rgb name="diffuseReflectance" value="0.6, 0.1, 0.1"/>
    <float name="alpha" value="0.2"/><string name="distribution" value="ggx"/></bsdf>
  <sensor type="perspective">
    <float name="fov" value="40"/><string name="fovAxis" value="y"/>
    <transform name="toWorld"><scale x="-1"/><lookat origin="0, 1, -5" target="0, 1, 0" up="0, 1, 0"/></transform>
    <sampler type="independent"><integer name="sampleCount" value="8"/></sampler>
    <film type="hdrfilm"><integer name="width" value="$res"/><integer name="height" value="20"/></film>
  </sensor>
  <shape type="rectangle">
    <transform name="toWorld"><scale value="3"/><rotate x="1" angle="-90"/></transform>
    <bsdf type="diffuse"><spectrum name="reflectance" value="0.25"/></bsdf>
  </shape>
  <shape type="cube"><transform name="toWorld"><scale value="0.5"/><translate y="0.5"/></transform>
    <ref id="red"/></shape>
  <shape type="rectangle"><boolean name="flipNormals" value="true"/>
    <transform name="toWorld"><rotate x="1" angle="-90"/><translate y="3"/></transform>
    <emitter type="area"><rgb name="radiance" value="5, 4, 3"/></emitter></shape>
  <shape type="sphere"><point name="center" x="1.5" y="0.5" z="0"/><float name="radius" value="0.5"/>
    <bsdf type="dielectric"><string name="intIOR" value="diamond"/></bsdf></shape>
  <emitter type="constant"><spectrum name="radiance" value="0.1"/></emitter>
</scene>"""


def test_handwritten_scene_semantics(pg):
    out = pg.mitsuba_xml.load(SCENE, defines={"depth": 7}, sphere_res=(16, 8))
    sc = out.scene
    assert out.integrator_props == {"maxDepth": 7} and out.spp == 8
    assert (sc.camera.width, sc.camera.height) == (40, 20) and sc.mirror_x
    # fovAxis=y: tan(fx / 2) = tan(20 deg) * aspect
    assert abs(np.tan(np.radians(sc.camera.fov_x_deg) / 2) - np.tan(np.radians(20)) * 2) < 1e-5
    floor = sc.positions[sc.indices[sc.shapes[0].tri_begin:sc.shapes[0].tri_begin + 2]].reshape(-1, 3)
    assert np.allclose(floor[:, 1], 0, atol=1e-6) and np.allclose(np.abs(floor[:, [0, 2]]).max(), 3)
    # the floor's normal faces +y after rotate(x, -90) of the rectangle's +z
    assert np.allclose(sc.normals[sc.indices[sc.shapes[0].tri_begin]], [0, 1, 0], atol=1e-6)
    cube = sc.positions[sc.indices[sc.shapes[1].tri_begin:sc.shapes[1].tri_begin + sc.shapes[1].tri_count]]
    assert np.allclose(cube.reshape(-1, 3).min(0), [-0.5, 0, -0.5]) and np.allclose(cube.reshape(-1, 3).max(0), [0.5, 1, 0.5])
    light = sc.shapes[2]
    assert light.emitter == 0 and list(sc.emitters[0].radiance)[:3] == [5, 4, 3]
    assert np.allclose(sc.normals[sc.indices[light.tri_begin]], [0, -1, 0], atol=1e-6)  # flipNormals: faces down
    m_red = sc.materials[sc.shapes[1].material]
    assert m_red.type == pg.capi.PG_BSDF_ROUGHPLASTIC and abs(m_red.alpha_u - 0.2) < 1e-7
    glass = sc.materials[sc.shapes[3].material]
    assert abs(glass.int_ior - 2.419) < 1e-6 and abs(glass.ext_ior - 1.000277) < 1e-6
    assert sc.envmap is not None and np.allclose(sc._env_rgb, 0.1)
    assert sc.materials[sc.shapes[0].material].diffuse_reflectance[0] == pytest.approx(0.25)
    with pytest.raises(NotImplementedError):
        pg.mitsuba_xml.load('<scene><bsdf type="ward"/></scene>')


def test_ply_and_obj_readers(pg, tmp_path):
    X = pg.mitsuba_xml
    V = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0]], np.float32)
    hdr = ("ply\nformat binary_little_endian 1.0\nelement vertex 4\nproperty float x\nproperty float y\n"
           "property float z\nelement face 1\nproperty list uchar int vertex_indices\nend_header\n")
    with open(tmp_path / "q.ply", "wb") as f:
        f.write(hdr.encode())
        f.write(V.astype("<f4").tobytes())
        f.write(bytes([4]) + np.array([0, 1, 2, 3], "<i4").tobytes())
    Vp, Fp, Np = X._read_ply(str(tmp_path / "q.ply"))
    assert np.array_equal(Vp, V) and Fp.tolist() == [[0, 1, 2], [0, 2, 3]] and Np is None
    with open(tmp_path / "q.obj", "w") as f:
        f.write("v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nf 1 2 3 4\n")
    Vo, Fo, No = X._read_obj(str(tmp_path / "q.obj"))
    assert np.array_equal(Vo, V) and Fo.tolist() == [[0, 1, 2], [0, 2, 3]] and No is None
    N = X._vertex_normals(Vo, Fo)
    assert np.allclose(N, [0, 0, 1])


def _ser_mesh_v3(V, F, N=None, double=True):
    """One mesh in the version-3 .serialized layout, packed by hand (trimesh.cpp:175-252: header,
    then a zlib stream of flags, counts, positions, [normals], indices; no name in v3)."""
    import struct
    import zlib
    flags = (0x2000 if double else 0x1000) | (0x0001 if N is not None else 0)
    ft = "<f8" if double else "<f4"
    body = struct.pack("<IQQ", flags, len(V), len(F)) + np.asarray(V, ft).tobytes()
    if N is not None:
        body += np.asarray(N, ft).tobytes()
    body += np.asarray(F, "<u4").tobytes()
    return struct.pack("<HH", 0x041C, 0x0003) + zlib.compress(body)


def test_serialized_reader(pg, tmp_path):
    """TriMesh::loadCompressed (trimesh.cpp:175-294): v3 multi-mesh file with a u32 offset
    dictionary, f64 positions, normals; v4 round trip through write_serialized; shapeIndex and the
    det < 0 index swap of serialized.cpp:197-202 through the XML loader."""
    import struct
    X = pg.mitsuba_xml
    V0 = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float64)
    V1 = np.array([[0, 0, 1], [2, 0, 1], [2, 2, 1], [0, 2, 1]], np.float64)
    F1 = np.array([[0, 1, 2], [0, 2, 3]])
    N1 = np.tile([0.0, 0.0, 1.0], (4, 1))
    m0 = _ser_mesh_v3(V0, [[0, 1, 2]])
    m1 = _ser_mesh_v3(V1, F1, N1)
    blob = m0 + m1 + struct.pack("<III", 0, len(m0), 2)
    path = tmp_path / "two.serialized"
    path.write_bytes(blob)
    V, F, N = X.read_serialized(str(path), 0)
    assert np.array_equal(V, V0) and F.tolist() == [[0, 1, 2]] and N is None
    V, F, N = X.read_serialized(str(path), 1)
    assert np.array_equal(V, V1) and np.array_equal(F, F1) and np.array_equal(N, N1)
    with pytest.raises(ValueError):
        X.read_serialized(str(path), 2)
    bad = tmp_path / "bad.serialized"
    bad.write_bytes(struct.pack("<HH", 0x1C04, 3) + b"\0" * 16)
    with pytest.raises(ValueError):
        X.read_serialized(str(bad))
    # v4 (names, f32) round trip
    p4 = tmp_path / "four.serialized"
    X.write_serialized(str(p4), [(V0, [[0, 1, 2]], None, "tri"), (V1, F1, N1, "quad")])
    V, F, N = X.read_serialized(str(p4), 1)
    assert np.array_equal(V, V1) and np.array_equal(F, F1) and np.array_equal(N, N1)
    # through the loader: shapeIndex 1, mirrored toWorld -> idx[0] <-> idx[1], normals (0, 0, 1) kept
    # (the mirror is along x, so the inverse-transpose leaves z normals unchanged)
    xml = ('<scene version="0.5.0"><shape type="serialized"><string name="filename" value="two.serialized"/>'
           '<integer name="shapeIndex" value="1"/><transform name="toWorld"><scale x="-1"/></transform></shape>'
           '</scene>')
    (tmp_path / "s.xml").write_text(xml)
    sc = X.load(str(tmp_path / "s.xml")).scene
    assert len(sc.shapes) == 1 and sc.shapes[0].tri_count == 2
    assert np.array_equal(sc._pos[0].astype(np.float64), V1 * [-1, 1, 1])
    assert sc._idx[0].tolist() == [[1, 0, 2], [2, 0, 3]]
    assert np.allclose(sc._nrm[0], N1)
