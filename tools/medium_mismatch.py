"""Where do the GPU's and the oracle's Woodcock free-flight distances differ on identical draws?
Runs test_gpu_volume.test_phase_and_medium_units' tracking inputs through both sides (global majorant,
free flight) and, for every ray whose distance differs, recomputes the density-box clip in float32
(numpy) and reports whether the entry distance t0, the first step or a later one differs.
usage (GPU box): python tools/medium_mismatch.py OUT.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import pgload  # noqa: E402
import oracle_py as O  # noqa: E402
from test_volume import _vol_cfg  # noqa: E402


def main(out):
    pg = pgload.load()
    O.build()
    from mitsuba_path_guiding_amd.integrator import Device
    sc = pg.scenes.smoke(16, 16, res=48)
    dev = Device(_vol_cfg(pg))
    dev.upload(sc)
    osc = O.OracleScene(pg.capi, sc)
    rng = np.random.default_rng(1)
    n = 100_000
    rng.normal(size=(n, 3)); rng.random((n, 2)); rng.normal(size=(n, 3)); rng.uniform(-1.1, 1.1, size=(n, 3))
    rays = np.zeros((n, 8), np.float32)
    rays[:, 0:3] = rng.uniform(-1.5, 1.5, size=(n, 3))
    d = rng.normal(size=(n, 3))
    rays[:, 4:7] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 7] = rng.uniform(0.5, 4.0, size=n)
    keys = rng.integers(0, 2 ** 32, size=(n, 2), dtype=np.uint32)
    gg = dev.medium_sample(0, rays, keys, transmittance=False, grid=False)
    cc = osc.medium_sample(0, rays, keys, transmittance=False, grid=False)
    diff = np.where(np.any(gg[:, :3] != cc[:, :3], axis=1))[0]
    print(f"{len(diff)} of {n} rays differ; same draw counts {np.mean(gg[:, 2] == cc[:, 2]):.5f}; "
          f"same hit flags {np.mean(gg[:, 0] == cc[:, 0]):.5f}")
    if len(diff):
        dt = np.abs(gg[diff, 1] - cc[diff, 1]) / np.maximum(np.abs(cc[diff, 1]), 1e-30)
        ulp = np.abs(gg[diff, 1].view(np.int32).astype(np.int64) - cc[diff, 1].view(np.int32).astype(np.int64))
        print("relative t difference quantiles 0.5/0.9/0.99/max", np.quantile(dt, [0.5, 0.9, 0.99, 1.0]))
        print("ulp difference histogram (1, 2, 3-8, >8):", [(ulp == 1).sum(), (ulp == 2).sum(),
              ((ulp >= 3) & (ulp <= 8)).sum(), (ulp > 8).sum()])
        print("rays starting inside [-1,1]^3 among the differing:",
              np.mean(np.all(np.abs(rays[diff, :3]) <= 1, axis=1)), "overall:", np.mean(np.all(np.abs(rays[:, :3]) <= 1, axis=1)))
    np.savez(out, rays=rays, keys=keys, gg=gg, cc=cc, diff=diff)
    dev.close()


if __name__ == "__main__":
    main(sys.argv[1])
