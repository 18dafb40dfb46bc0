"""Synthetic scene generators: deterministic, well-formed, and in the size classes of SURVEY.md §8."""
import numpy as np


def _check(sc):
    d = sc.desc()
    assert d.num_triangles == len(sc.indices) and d.num_vertices == len(sc.positions)
    assert sc.indices.max() < len(sc.positions)
    covered = np.zeros(d.num_triangles, int)
    for s in sc.shapes:
        covered[s.tri_begin: s.tri_begin + s.tri_count] += 1
        assert s.material < len(sc.materials)
    assert (covered == 1).all()
    assert len(sc.emitters) >= 1
    for e in sc.emitters:
        assert sc.shapes[e.shape].emitter >= 0
    assert np.isfinite(sc.positions).all() and np.isfinite(sc.normals).all()
    assert np.allclose(np.linalg.norm(sc.normals, axis=1), 1, atol=1e-4)


def test_cornell(pg):
    sc = pg.scenes.cornell(64, 48)
    _check(sc)
    assert sc.num_triangles == 32 and (sc.width, sc.height) == (64, 48)


def test_ajar_door_deterministic(pg):
    a = pg.scenes.ajar_door(64, 36)
    b = pg.scenes.ajar_door(64, 36)
    _check(a)
    assert np.array_equal(a.positions, b.positions) and np.array_equal(a.indices, b.indices)
    assert 10_000 <= a.num_triangles <= 100_000
    assert len(a.emitters) == 1  # the only light is in the far room
    kinds = {m.type for m in a.materials}
    assert {pg.capi.PG_BSDF_ROUGHCONDUCTOR, pg.capi.PG_BSDF_DIELECTRIC} <= kinds


def test_kitchen_size_class(pg):
    sc = pg.scenes.kitchen(64, 36, target_tris=150_000)
    _check(sc)
    assert sc.num_triangles >= 150_000 and len(sc.emitters) >= 4
