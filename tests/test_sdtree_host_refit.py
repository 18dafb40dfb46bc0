"""The library's host refit (pg_sdtree.cpp, what pg_refit runs) against the oracle's refit on the same
building statistics, on the CPU: the same serialized tree in, the same tree out -- including the
learned BSDF-sampling fractions (PG_FRACTION_LEARNED).  The library code is compiled here from its
source through a test-only shim (tests/csrc/sdtree_shim.cpp)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def shim(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("shim") / "libsdshim.so")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-pthread", "-o", out,
                           os.path.join(ROOT, "tests", "csrc", "sdtree_shim.cpp"),
                           os.path.join(ROOT, "mitsuba-path-guiding_amd", "csrc", "pg_sdtree.cpp")])
    L = C.CDLL(out)
    L.shim_refit.restype = C.c_int
    L.shim_refit.argtypes = [C.c_void_p, C.c_size_t, C.c_uint32, C.c_float, C.c_float, C.c_int, C.c_int, C.c_void_p,
                             C.c_size_t, C.POINTER(C.c_size_t)]
    return L


def host_refit(L, blob, it, cfg, learn):
    blob = np.ascontiguousarray(blob, np.uint8)
    n = C.c_size_t()
    assert L.shim_refit(blob.ctypes.data, len(blob), it, cfg.s_tree_threshold, cfg.d_tree_threshold,
                        cfg.d_tree_max_depth, int(learn), None, 0, C.byref(n)) == 0
    out = np.zeros(n.value, np.uint8)
    assert L.shim_refit(blob.ctypes.data, len(blob), it, cfg.s_tree_threshold, cfg.d_tree_threshold,
                        cfg.d_tree_max_depth, int(learn), out.ctypes.data, len(out), C.byref(n)) == 0
    return out


@pytest.mark.parametrize("mode", ["fixed", "learned"])
def test_host_refit_equals_oracle(pg, O, shim, mode):
    bound = pg.capi.PG_FRACTION_LEARNED if mode == "learned" else pg.capi.PG_FRACTION_FIXED
    sc = pg.scenes.cornell(48, 48)
    cfg = pg.capi.default_config(guiding=1, s_tree_threshold=400.0, bsdf_fraction_bound=bound)
    osc = O.OracleScene(pg.capi, sc)
    tree = O.OracleSDTree(osc)
    off = 0
    for it in range(4):
        O.render(osc, cfg, 2 ** it, off, record=True, sdtree=tree, nthreads=4)
        off += 2 ** it
        tree.splat_pending()
        before = tree.serialize()
        tree.refit(it, cfg)
        assert np.array_equal(host_refit(shim, before, it, cfg, mode == "learned"), tree.serialize()), it
