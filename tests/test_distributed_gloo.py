"""World-size-2 and -4 (C4's rank count) gloo tests of the multi-rank training path (CPU): tile sharding + the exchange of
mitsuba_path_guiding_amd.distributed (both the building-statistics all-reduce and the record
all-gather) + refit must leave every rank with the same SD-tree, bit for bit, and that tree must
equal a single-rank training on the whole image (splats are exact fixed-point arithmetic, so
neither record order nor where the sums were formed can matter).

The per-rank "device" here is a CPU stand-in built on the oracle (test double): the exchange code
under test only needs the Device interface it calls (record_count / get_records / splat_records /
splat_local / tree_stats_words / get_tree_stats / put_tree_stats).  The stand-in reads and writes
the building statistics through the tree's wire format (pg_sdtree.cpp serialize), in the same
order as pg_get_tree_stats.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RES, ITERS, THR = 48, 3, 300.0


def tile_shard(W, H, rank, world, T=32):
    """pg_upload_scene's shard: 32x32 tiles dealt round-robin, row-major inside a tile."""
    tx, ty = (W + T - 1) // T, (H + T - 1) // T
    pix = []
    for t in range(tx * ty):
        if t % world != rank:
            continue
        x0, y0 = (t % tx) * T, (t // tx) * T
        for y in range(y0, min(y0 + T, H)):
            for x in range(x0, min(x0 + T, W)):
                pix.append(y * W + x)
    return np.array(pix, np.uint32)


class OracleShardDevice:
    def __init__(self, pg, O, scene, cfg, rank, world):
        self.pg, self.O, self.cfg = pg, O, cfg
        self.osc = O.OracleScene(pg.capi, scene)
        self.tree = O.OracleSDTree(self.osc)
        self.pixels = tile_shard(scene.width, scene.height, rank, world)
        self.pending = np.zeros(0, np.uint8)

    def render_pass(self, spp, offset, record):
        self.O.render(self.osc, self.cfg, spp, offset, record=record, sdtree=self.tree, pixels=self.pixels,
                      nthreads=1)
        self.pending = self.tree.take_records(self.pg.capi)

    def record_count(self):
        return len(self.pending) // 32

    def get_records(self, dst_ptr=None, max_records=None):
        assert dst_ptr is None
        return self.pending

    def splat_records(self, recs=None, device_ptr=None, count=None):
        self.tree.splat_bytes(recs)

    def refit(self, it):
        self.tree.refit(it, self.cfg)
        self.pending = np.zeros(0, np.uint8)

    def splat_local(self):
        self.tree.splat_bytes(self.pending)

    # building statistics through the wire format (v2): header 16 B, box 32 B, counts (snodes,
    # dtrees, sampling nodes, building nodes), snodes 8 B, D-tree meta 32 B (record count at word 5),
    # sampling nodes 32 B, building nodes 48 B (u64 sum[4] + u32 child[4]), then FRAC u64 learned-
    # fraction statistics per D-tree -- pg_get_tree_stats' order: sums, counts, fraction statistics
    FRAC = 11

    def _layout(self, blob):
        ns, nd, nsamp, nb = np.frombuffer(blob[48:64].tobytes(), np.uint32)
        meta = 64 + 8 * int(ns)
        build = meta + 32 * int(nd) + 32 * int(nsamp)
        return int(nd), int(nb), meta, build

    def tree_stats_words(self):
        nd, nb, _, _ = self._layout(self.tree.serialize())
        return 4 * nb + nd + self.FRAC * nd

    def get_tree_stats(self):
        blob = self.tree.serialize()
        nd, nb, meta, build = self._layout(blob)
        sums = np.frombuffer(blob[build:build + 48 * nb].tobytes(), np.uint8).reshape(nb, 48)[:, :32]
        cnt = np.frombuffer(blob[meta:meta + 32 * nd].tobytes(), np.uint32).reshape(nd, 8)[:, 5]
        frac = np.frombuffer(blob[build + 48 * nb:].tobytes(), np.uint64)
        assert len(frac) == self.FRAC * nd
        return np.concatenate([sums.copy().view(np.uint64).reshape(-1), cnt.astype(np.uint64), frac])

    def put_tree_stats(self, stats):
        blob = np.array(self.tree.serialize(), np.uint8)
        nd, nb, meta, build = self._layout(blob)
        stats = np.asarray(stats, np.uint64)
        b = blob[build:build + 48 * nb].reshape(nb, 48)
        b[:, :32] = stats[:4 * nb].reshape(nb, 4).view(np.uint8)
        m = blob[meta:meta + 32 * nd].reshape(nd, 32)
        m[:, 20:24] = stats[4 * nb:4 * nb + nd].astype(np.uint32).reshape(nd, 1).view(np.uint8)
        blob[build + 48 * nb:] = stats[4 * nb + nd:].view(np.uint8)
        self.tree.deserialize(blob)


def _worker(rank, world, port, outdir, mode):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import pgload
    import oracle_py as O
    pg = pgload.load()
    from mitsuba_path_guiding_amd import distributed as D
    D.init("gloo")
    sc = pg.scenes.cornell(RES, RES)
    cfg = pg.capi.default_config(guiding=1, s_tree_threshold=THR, rank=rank, world_size=world)
    dev = OracleShardDevice(pg, O, sc, cfg, rank, world)
    exchange = D.make_exchange(on_device=False, mode=mode)
    off = 0
    for it in range(ITERS):
        dev.render_pass(2 ** it, off, True)
        off += 2 ** it
        counts = exchange(dev)
        assert len(counts) == world
        dev.refit(it)
    np.save(os.path.join(outdir, f"tree{rank}.npy"), dev.tree.serialize())
    # final render of the shard with the trained tree, films summed to rank 0 (distributed.reduce_film)
    rgbw, sq = O.render(dev.osc, cfg, 4, off, sdtree=dev.tree, pixels=dev.pixels, nthreads=1)[:2]
    rgbw, sq = D.reduce_film(rgbw, sq, on_device=False)
    if rank == 0:
        np.save(os.path.join(outdir, "film.npy"), np.stack([rgbw, sq]))
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode,world", [("allreduce", 2), ("allgather", 2), ("allreduce", 4)])
def test_multi_rank_exchange_gives_identical_trees(pg, O, tmp_path, mode, world):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), mode), nprocs=world, join=True)
    t0 = np.load(tmp_path / "tree0.npy")
    for r in range(1, world):
        assert np.array_equal(t0, np.load(tmp_path / f"tree{r}.npy"))
    # single rank over the whole image, same sample indices -> same record multiset -> same tree
    sc = pg.scenes.cornell(RES, RES)
    cfg = pg.capi.default_config(guiding=1, s_tree_threshold=THR)
    osc = O.OracleScene(pg.capi, sc)
    tree = O.OracleSDTree(osc)
    off = 0
    for it in range(ITERS):
        O.render(osc, cfg, 2 ** it, off, record=True, sdtree=tree, nthreads=2)
        off += 2 ** it
        tree.splat_pending()
        tree.refit(it, cfg)
    assert np.array_equal(tree.serialize(), t0)
    # the reduced film equals the single-rank film bit for bit (disjoint tiles, one contributor each)
    film = np.load(tmp_path / "film.npy")
    rgbw, sq = O.render(osc, cfg, 4, off, sdtree=tree, nthreads=2)[:2]
    assert np.array_equal(film[0], rgbw) and np.array_equal(film[1], sq)


def test_shard_covers_image_once():
    W, H = 100, 70
    parts = [tile_shard(W, H, r, 3) for r in range(3)]
    allp = np.concatenate(parts)
    assert len(allp) == W * H and len(np.unique(allp)) == W * H


class _SleepDevice:
    """Stand-in for the render-time test: a pass of spp samples takes spp x `per_spp` seconds."""

    def __init__(self, per_spp):
        self.per_spp = per_spp
        self.spp = 0

    def render_pass(self, spp, offset, record=False):
        import time
        time.sleep(spp * self.per_spp)
        self.spp += spp


def _render_time_worker(rank, world, port, outdir):
    sys.path.insert(0, ROOT)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import pgload
    pg = pgload.load()
    from mitsuba_path_guiding_amd import distributed as D
    from mitsuba_path_guiding_amd.integrator import ProgressivePathTracer
    import time
    D.init("gloo")
    t = ProgressivePathTracer({"maxRenderTime": 0.6, "samplesPerProgression": 2}, rank=rank, world_size=world,
                              reduce_sum=D.make_reduce_sum(False))
    t.dev = _SleepDevice(0.002 * (1 + 3 * rank))  # rank 1 is 4x slower: its clock must rule
    t0 = time.perf_counter()
    done = t._render_time_sharded(t0)
    np.save(os.path.join(outdir, f"rt{rank}.npy"), np.array([done, t.dev.spp, time.perf_counter() - t0]))
    import torch.distributed as dist
    dist.destroy_process_group()


def test_max_render_time_sharded_ranks_agree(tmp_path):
    """maxRenderTime with a tile shard: every rank renders the same number of whole progressions,
    sized by the slowest rank's clock, and the budget holds (per-rank clocks left the
    reduced image with tile-dependent sample counts)."""
    import torch.multiprocessing as mp
    mp.spawn(_render_time_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0, r1 = np.load(tmp_path / "rt0.npy"), np.load(tmp_path / "rt1.npy")
    assert r0[0] == r1[0] == r0[1] == r1[1] > 0 and r0[0] % 2 == 0
    assert r1[2] < 0.6 * 1.6 + 0.2  # overshoot below about half the budget plus one progression
