"""Conductor eta / k: the RGB values of every preset are derived from the reference's spectral data
(data/ior/*.spd, Spectrum::fromContinuousSpectrum in the RGB build, roughconductor.cpp:173-188) by
tests/golden/make_conductor_fixture.py.  Pins: the derivation reproduces the RGB values Mitsuba's
RGB build reports for Cu / Al / Au to 6 digits; the package table equals the fixture; the XML
loader resolves presets and extEta as roughconductor does."""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

# RGB eta / k that Mitsuba 0.5's RGB build prints for its Cu, Al and Au presets (the values the
# previous hard-coded table held)
MITSUBA_RGB = {
    "Cu": ((0.200438, 0.924033, 1.10221), (3.91295, 2.45285, 2.14219)),
    "Al": ((1.65746, 0.880369, 0.521229), (9.22387, 6.26952, 4.83700)),
    "Au": ((0.143119, 0.374957, 1.44248), (3.98316, 2.38572, 1.60322)),
}


def fixture():
    return json.load(open(os.path.join(HERE, "golden", "conductor_rgb.json")))["materials"]


def test_fixture_reproduces_mitsuba_rgb():
    f = fixture()
    for name, (eta, k) in MITSUBA_RGB.items():
        np.testing.assert_allclose(f[name]["eta"], eta, rtol=2e-5, atol=1e-6)
        np.testing.assert_allclose(f[name]["k"], k, rtol=2e-5, atol=1e-6)
    assert len(f) >= 60  # every preset with both an eta and a k file


def test_package_table_is_the_fixture(pg):
    f = fixture()
    assert set(pg.scenes.CONDUCTORS) == set(f)
    for name, (eta, k) in pg.scenes.CONDUCTORS.items():
        assert list(eta) == f[name]["eta"] and list(k) == f[name]["k"]


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "data", "ior")), reason="reference tree not present")
def test_fixture_regenerates_from_reference_spectra(tmp_path):
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_conductor_fixture as M
    cie = M.cie_tables(REF)
    f = fixture()
    for name in ("Cu", "Ag", "Cr", "W"):
        base = os.path.join(REF, "data", "ior", name)
        eta = M.to_rgb(M.read_spd(base + ".eta.spd"), cie)
        k = M.to_rgb(M.read_spd(base + ".k.spd"), cie)
        np.testing.assert_allclose(eta, f[name]["eta"], atol=2e-6)
        np.testing.assert_allclose(k, f[name]["k"], atol=2e-6)


def test_xml_conductor_presets(pg):
    f = fixture()
    xml = """<scene version="0.5.0">
      <sensor type="perspective"><float name="fov" value="40"/>
        <transform name="toWorld"><lookat origin="0,0,-3" target="0,0,0" up="0,1,0"/></transform>
        <film type="hdrfilm"><integer name="width" value="8"/><integer name="height" value="8"/></film></sensor>
      <shape type="rectangle"><bsdf type="roughconductor"><string name="material" value="Ag"/></bsdf></shape>
      <shape type="rectangle"><bsdf type="conductor"><string name="material" value="Cr"/>
        <float name="extEta" value="1.5"/></bsdf></shape>
    </scene>"""
    x = pg.mitsuba_xml.load(xml)
    m0, m1 = x.scene.materials[0], x.scene.materials[1]
    np.testing.assert_allclose(list(m0.eta[:3]), f["Ag"]["eta"], rtol=1e-6)
    np.testing.assert_allclose(list(m0.k[:3]), f["Ag"]["k"], rtol=1e-6)
    np.testing.assert_allclose(list(m1.eta[:3]), np.array(f["Cr"]["eta"]) / 1.5, rtol=1e-6)
    np.testing.assert_allclose(list(m1.k[:3]), np.array(f["Cr"]["k"]) / 1.5, rtol=1e-6)
    with pytest.raises(ValueError):
        pg.mitsuba_xml.load(xml.replace('"Ag"', '"Unobtainium"'))
