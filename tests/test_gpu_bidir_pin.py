"""GPU radiance loops pinned by the reference's analytic two-disk scenes (tests/test_bidir_pin.py has
the fixture and the oracle side): the surface wavefront (k_camera / k_trace / k_shade / k_rays /
k_film) on test_bidir_0, the volumetric path (the default wavefront: k_vcam / k_vflight / k_vvertex /
k_vtail) on test_bidir_0 and test_bidir_2,
each per pixel and on the image mean against the float64 quadrature; and the guided surface path
(SD-tree trained on the GPU) against the same analytic image (guiding is unbiased)."""
import numpy as np
import pytest

from test_bidir_pin import PIN_CASES, bidir_scene, check, expected_image

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,nee,exact,key", PIN_CASES)
def test_gpu_pinned_by_bidir_scene(pg, name, nee, exact, key):
    from mitsuba_path_guiding_amd.integrator import ProgressivePathTracer, ProgressiveVolumetricPathTracer
    sc, _ = bidir_scene(pg, name)
    T = ProgressiveVolumetricPathTracer if name == "bidir_2" else ProgressivePathTracer
    spp = 4096 if nee else 16384
    t = T({"useNee": bool(nee), "samplesPerProgression": spp, "exactMis": bool(exact)})
    t.preprocess(sc)
    rgbw, sq = t.render(spp)
    t.postprocess()
    zmean, rel = check(rgbw, sq, expected_image(key), spp)
    print(f"gpu {name} nee={nee} exact={exact}: image mean {rel:+.2e} relative to {key}, z = {zmean:+.2f}")
    assert abs(rel) < 5e-3


def test_gpu_volpath_on_surface_scene_pinned(pg):
    """The volumetric megakernel on the medium-free scene (its surface branch)."""
    from mitsuba_path_guiding_amd.integrator import ProgressiveVolumetricPathTracer
    sc, expected = bidir_scene(pg, "bidir_0")
    t = ProgressiveVolumetricPathTracer({"samplesPerProgression": 4096})
    t.preprocess(sc)
    rgbw, sq = t.render(4096)
    t.postprocess()
    zmean, rel = check(rgbw, sq, expected, 4096)
    assert abs(rel) < 5e-3


def test_gpu_guided_pinned_by_bidir_0(pg):
    from mitsuba_path_guiding_amd.integrator import GuidedPathTracer
    sc, expected = bidir_scene(pg, "bidir_0")
    t = GuidedPathTracer({"trainingIterations": 5, "sTreeThreshold": 400.0, "samplesPerProgression": 4096})
    t.preprocess(sc)
    rgbw, sq = t.render(4096)
    st = t.postprocess()
    assert st["records"] > 0
    zmean, rel = check(rgbw, sq, expected, 4096)
    assert abs(rel) < 5e-3
