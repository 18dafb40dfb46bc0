"""Regenerates the committed golden fixtures (run in the build container; the GPU box never needs it).

  bunny.npz          positions/faces of the reference's data/tests/bunny.ply (35,947 vertices,
                     69,451 faces) — the ray-cast workload of src/tests/test_kd.cpp:86-130.  Data only.
  sdtree_cornell.npz SD-tree golden vectors from the CPU oracle (parity UNPINNED against the reference,
                     which has no guiding code): the serialized tree after 3 guided training
                     iterations on a 32x32 Cornell box, and pdf/sample queries on it.
  film_cornell.npz   oracle film (32x32, 16 spp, unguided) pinning the oracle's own determinism.
dgeom_kat.json is transcribed by hand from src/tests/test_dgeom.cpp:36-121.

usage: python tests/golden/make_fixtures.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
REF_BUNNY = "/root/reference/data/tests/bunny.ply"


def read_ply_binary(path):
    with open(path, "rb") as f:
        header = []
        while True:
            line = f.readline().decode("ascii").strip()
            header.append(line)
            if line == "end_header":
                break
        nv = int([h for h in header if h.startswith("element vertex")][0].split()[-1])
        nf = int([h for h in header if h.startswith("element face")][0].split()[-1])
        assert "format binary_little_endian 1.0" in header
        V = np.frombuffer(f.read(nv * 12), dtype="<f4").reshape(nv, 3).copy()
        rec = np.dtype([("n", "u1"), ("i", "<i4", (3,))])
        F = np.frombuffer(f.read(nf * rec.itemsize), dtype=rec, count=nf)
        assert (F["n"] == 3).all()
        return V, F["i"].astype(np.uint32)


def sdtree_queries(seed=5, n=4096):
    rng = np.random.default_rng(seed)
    pos = rng.random((n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    u = rng.random((n, 2)).astype(np.float32)
    return pos, d, u


def main():
    if os.path.exists(REF_BUNNY):
        V, F = read_ply_binary(REF_BUNNY)
        np.savez_compressed(os.path.join(HERE, "bunny.npz"), positions=V, faces=F)
        print("bunny", V.shape, F.shape)
    import pgload
    import oracle_py as O
    pg = pgload.load()
    O.build()
    sc = pg.scenes.cornell(32, 32)
    osc = O.OracleScene(pg.capi, sc)
    # Mueller et al.'s fixed BSDF fraction (the fixture predates pg_config.bsdf_fraction_bound)
    cfg = pg.capi.default_config(guiding=1, s_tree_threshold=400.0, bsdf_fraction_bound=pg.capi.PG_FRACTION_FIXED)
    tree = O.OracleSDTree(osc)
    for it in range(3):
        O.render(osc, cfg, 2 ** it, 2 ** it - 1, record=True, sdtree=tree, nthreads=1)
        tree.splat_pending()
        tree.refit(it, cfg)
    blob = tree.serialize()
    lo, hi = sc.bounds()
    pos, d, u = sdtree_queries()
    pos = lo + (hi - lo) * pos
    pdf = tree.pdf(pos, d)
    sd, spdf = tree.sample(pos, u)
    np.savez_compressed(os.path.join(HERE, "sdtree_cornell.npz"), blob=blob, pos=pos, dir=d, u=u, pdf=pdf,
                        sample_dir=sd, sample_pdf=spdf)
    print("sdtree blob", len(blob), "bytes")
    rgbw, sq, st = O.render(osc, pg.capi.default_config(), 16, 0, nthreads=1)
    np.savez_compressed(os.path.join(HERE, "film_cornell.npz"), rgbw=rgbw, sumsq=sq, stats=st)
    print("film", rgbw[..., :3].mean())


if __name__ == "__main__":
    main()
