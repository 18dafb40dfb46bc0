"""Small GPU timing run: one unguided pass over cornell and ajar (development helper)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pgload
pg = pgload.load()
from mitsuba_path_guiding_amd.integrator import Device

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 4
lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 0
for name, sc in [("cornell", pg.scenes.cornell(512, 512)), ("ajar", pg.scenes.ajar_door(1280, 720))]:
    d = Device(pg.capi.default_config(path_lanes=lanes, kernel_timing=1))
    d.upload(sc)
    d.render_pass(1, 0)
    t = time.time(); d.render_pass(spp, 1); dt = time.time() - t
    st = d.stats()
    n = sc.width * sc.height * spp
    print(name, f"{n/dt/1e6:.1f} Mpaths/s wall {dt*1e3:.1f} ms, seg/path {st['segments']/st['paths']:.2f}, "
          f"trace {st['trace_ms']:.1f} shade {st['shade_ms']:.1f} shadow {st['shadow_ms']:.1f} ms", flush=True)
    d.close()
