"""The C-ABI library (mitsuba-path-guiding_amd/build/libpgamd.so) loads, exports every entry point
include/pg_capi.h declares, and its struct layouts match the ctypes mirror.  No compute happens
here (CPU-only container): pg_create must fail cleanly with PG_ERR_NO_DEVICE."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pg_capi.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:pg_status|const char \*|int32_t)\s*\*?\s*(pg_\w+)\s*\(", src, re.M)))


def test_header_and_mirror_agree(pg):
    decl = declared_functions()
    mirrored = sorted(n for n, _, _ in pg.capi.SIGNATURES)
    assert decl == mirrored
    assert len(decl) >= 20


def test_library_exports_every_symbol(pg):
    lib = pg.capi.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", pg.capi.LIB_PATH], capture_output=True, text=True).stdout
    for name in declared_functions():
        assert re.search(rf"\bT {name}\b", out), name
    assert lib.pg_abi_version() == pg.capi.PG_ABI_VERSION == 12


def test_struct_layouts_match_header(pg):
    """Compile a probe against the header with gcc and compare sizeof/offsetof with ctypes."""
    c = pg.capi
    structs = {"pg_material": c.pg_material, "pg_shape": c.pg_shape, "pg_emitter": c.pg_emitter,
               "pg_camera": c.pg_camera, "pg_scene_desc": c.pg_scene_desc, "pg_config": c.pg_config,
               "pg_record": c.pg_record, "pg_stats": c.pg_stats, "pg_medium": c.pg_medium,
               "pg_envmap": c.pg_envmap}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for s, cls in structs.items():
        lines.append(f'printf("{s} %zu\\n", sizeof({s}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{s}.{f} %zu\\n", offsetof({s}, {f}));')
    lines.append("return 0; }")
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "probe.c")
        exe = os.path.join(d, "probe")
        open(src, "w").write("\n".join(lines))
        subprocess.check_call(["gcc", "-std=c99", "-o", exe, src])
        got = dict(l.split() for l in subprocess.check_output([exe], text=True).splitlines())
    for s, cls in structs.items():
        assert int(got[s]) == C.sizeof(cls), s
        for f, _ in cls._fields_:
            assert int(got[f"{s}.{f}"]) == getattr(cls, f).offset, (s, f)
    assert C.sizeof(c.pg_record) == 32
    assert C.sizeof(c.pg_material) == 112


def test_default_config_matches_library(pg):
    lib = pg.capi.load_library()
    a = pg.capi.pg_config()
    assert lib.pg_config_default(C.byref(a)) == 0
    b = pg.capi.default_config()
    assert bytes(a) == bytes(b)


def test_create_without_device_fails_cleanly(pg):
    lib = pg.capi.load_library()
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is visible")
    except ImportError:
        pass
    h = C.c_void_p()
    cfg = pg.capi.default_config()
    st = lib.pg_create(C.byref(cfg), C.byref(h))
    assert st == pg.capi.PG_ERR_NO_DEVICE
    assert b"no HIP device" in lib.pg_last_error(None)
    assert h.value is None
    bad = pg.capi.default_config(rank=3, world_size=2)
    assert lib.pg_create(C.byref(bad), C.byref(h)) == pg.capi.PG_ERR_INVALID
    assert lib.pg_destroy(None) == 0
    assert lib.pg_cancel(None) == pg.capi.PG_ERR_INVALID


def test_integrator_props_map_to_config(pg):
    from mitsuba_path_guiding_amd.integrator import GuidedPathTracer
    g = GuidedPathTracer({"maxDepth": 8, "rrDepth": 3, "useNee": False, "hideEmitters": True,
                          "sTreeThreshold": 4000, "dTreeThreshold": 0.02, "bsdfSamplingFraction": 0.3,
                          "trainingIterations": 7, "samplesPerProgression": 4}, rank=1, world_size=4)
    c = g.cfg
    assert (c.max_depth, c.rr_depth, c.use_nee, c.hide_emitters) == (8, 3, 0, 1)
    assert c.guiding == 1 and abs(c.bsdf_sampling_fraction - 0.3) < 1e-7
    assert (c.rank, c.world_size) == (1, 4)
    assert g.training_iterations == 7 and g.spp_per_progression == 4
