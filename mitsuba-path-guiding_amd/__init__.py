"""MI355X-native guided path-tracing integrator (drop-in for the hot path of the Mitsuba
progressive path integrator).  See DESIGN.md.  Import through pgload.load()."""
from . import capi, scenes, integrator, mitsuba_xml  # noqa: F401
