"""The Mitsuba plugin adapter (mitsuba_plugin/, unbuildable here: it needs the fork's Boost-based
headers) only calls entry points include/pg_capi.h declares, checks every pg_status, and covers the
postprogression exchanges, the environment emitter and participating media."""
import os
import re

from test_capi_abi import declared_functions

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "mitsuba_plugin", f) for f in ("guided_gpu.h", "guided_gpu.cpp", "guided_gpu_volpath.cpp")]


def adapter_text():
    """The adapter's code without // comments."""
    return "\n".join(re.sub(r"//.*", "", open(p).read()) for p in SRC)


def test_adapter_calls_only_declared_entry_points():
    calls = set(re.findall(r"\b(pg_[a-z0-9_]+)\s*\(", adapter_text()))
    assert calls <= set(declared_functions()), calls - set(declared_functions())
    for needed in ("pg_create", "pg_upload_scene", "pg_render_pass", "pg_render_time", "pg_splat_local_records",
                   "pg_refit", "pg_comm_allreduce_tree_stats", "pg_comm_allgather_records", "pg_comm_reduce_film",
                   "pg_comm_allreduce_f64", "pg_read_film", "pg_reset_film", "pg_cancel", "pg_destroy"):
        assert needed in calls, needed


def test_every_status_is_checked():
    """Each pg_ call is wrapped in check(...), assigned to a pg_status, or is pg_cancel/pg_destroy/
    pg_last_error/pg_config_default (no status to act on)."""
    text = adapter_text()
    for m in re.finditer(r"\b(pg_[a-z0-9_]+)\s*\(", text):
        name = m.group(1)
        if name in ("pg_cancel", "pg_destroy", "pg_last_error", "pg_config_default"):
            continue
        line = text[text.rfind("\n", 0, m.start()) + 1: text.find("\n", m.start())]
        assert re.search(r"check\(\s*" + name, line) or re.search(r"pg_status \w+ =|== PG_OK|st = ", line), line


def test_adapter_flattens_env_and_media():
    t = adapter_text()
    assert "getEnvironmentEmitter" in t and "desc.envmap" in t and "ConstantBackgroundEmitter" in t
    assert "getInteriorMedium" in t and "getExteriorMedium" in t and "camera_medium" in t
    assert "PG_INTEGRATOR_VOLPATH" in t and "HGPhaseFunction" in t


def test_adapter_feeds_denoiser_and_combines_iterations():
    """INTEGRATION.md's promises: with `denoise` or `denoiserFile` the adapter reads pg_read_aovs and feeds the per-pixel means
    to the fork's Denoiser (denoiser.cpp:138-144, Denoiser::add / denoise); `sampleCombination =
    "inversevar"` keeps every training iteration's film (pg_read_film + pg_reset_film) and combines them
    with inverse-variance weights all-reduced over ranks."""
    t = adapter_text()
    aov = t[t.index("if (m_cfg.aovs && (m_denoise"):]
    assert "pg_read_aovs" in aov and "Denoiser" in aov and "->add(" in aov and "->denoise()" in aov
    assert '"sampleCombination"' in t and '"inversevar"' in t
    train = t[t.index("for (int it = 0; it < m_trainingIterations"):t.index("pg_render_time")]
    assert "pg_read_film" in train and "pg_reset_film" in train
    comb = t[t.index("void combineInverseVariance"):]
    assert "pg_comm_allreduce_f64" in comb[:comb.index("for (size_t i = 0; i < npix; ++i) {\n            double")]
