"""CPU ground truth for the bench's GPU/CPU RMSE comparison (bench.py cpu_baseline):
the unguided ORACLE path tracer (independent of the GPU and of guiding) at 8192 spp, seed 4242, on
the 64 tiles of 32x32 starting at the bench's centre tile of C3 (ajar_door 1280x720).  The bench's
CPU sample takes its tiles from the same start, so every tile it renders is covered while it renders
at most 64.  Writes tests/golden/c3_cpu_gt_tiles.npz (pixel ids + f32 mean radiance).

usage: python tests/golden/make_c3_cpu_gt.py [--spp 8192] [--tiles 64] [--threads N]"""
import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def bench_tiles(width, height, T=32):
    """bench.py cpu_baseline's tile list (row-major 32x32 tiles) and its start index."""
    tiles = [[y * width + x for y in range(ty, min(ty + T, height)) for x in range(tx, min(tx + T, width))]
             for ty in range(0, height, T) for tx in range(0, width, T)]
    return tiles, len(tiles) // 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=8192)
    ap.add_argument("--tiles", type=int, default=64)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--out", default=os.path.join(HERE, "c3_cpu_gt_tiles.npz"))
    a = ap.parse_args()
    import pgload
    import oracle_py as O
    pg = pgload.load()
    sc = pg.scenes.ajar_door(1280, 720)
    tiles, mid = bench_tiles(sc.width, sc.height)
    pix = np.array([p for i in range(a.tiles) for p in tiles[(mid + i) % len(tiles)]], np.uint32)
    osc = O.OracleScene(pg.capi, sc)
    cfg = pg.capi.default_config(seed=4242)
    film = (np.zeros((sc.height, sc.width, 4), np.float32), np.zeros((sc.height, sc.width, 4), np.float32))
    t0 = time.time()
    step = 512
    for k in range(0, a.spp, step):  # batches: float sums stay well conditioned, progress is visible
        O.render(osc, cfg, min(step, a.spp - k), k, pixels=pix, nthreads=a.threads, film=film)
        print(f"{k + step} spp, {time.time() - t0:.0f} s", flush=True)
    rgbw = film[0].reshape(-1, 4)[pix]
    mean = rgbw[:, :3] / np.maximum(rgbw[:, 3:], 1)
    np.savez_compressed(a.out, pixels=pix, mean=mean.astype(np.float32), spp=np.int64(a.spp), seed=np.int32(4242),
                        integrator=np.bytes_(b"oracle unguided progressive path tracer (CPU)"))
    print("wrote", a.out, mean.shape, float(mean.mean()))


if __name__ == "__main__":
    main()
