"""The library's own multi-GPU path (pg_comm_*: one RCCL communicator per context, the C++ adapter's
exchange, include/pg_capi.h) on the one GPU of the test box: a single-rank communicator must leave
training, tree and film exactly as the communicator-free path leaves them.  (RCCL refuses two ranks
on one device, so the multi-rank exchange arithmetic is covered by the gloo tests and by
test_tree_stats_allreduce_equals_single_rank; bench.py --exchange capi runs it on N GPUs.)"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _train(pg, sc, comm, mode="allreduce"):
    from mitsuba_path_guiding_amd.integrator import Device
    d = Device(pg.capi.default_config(guiding=1, s_tree_threshold=200.0))
    d.upload(sc)
    if comm:
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")  # single-host bootstrap
        d.comm_init(d.comm_unique_id())
    off = 0
    for it in range(3):
        d.render_pass(2 ** it, off, record=True)
        off += 2 ** it
        if comm and mode == "allgather":  # pg_comm_allgather_records: gather + splat of every rank's records
            n = d.record_count()
            assert d.comm_allgather_records() == [n] and n > 0
        else:
            d.splat_local()
        if comm and mode == "allreduce":
            before = d.get_tree_stats()
            d.comm_allreduce_tree_stats()
            assert np.array_equal(before, d.get_tree_stats())
        d.refit(it)
    d.render_pass(8, off)
    film = d.read_film()
    if comm:
        d.comm_reduce_film(0)
        again = d.read_film()
        assert np.array_equal(film[0], again[0]) and np.array_equal(film[1], again[1])
        assert np.array_equal(d.comm_allreduce_f64([1.5, -2.0, 3.25]), [1.5, -2.0, 3.25])
    tree = d.get_sdtree()
    d.close()
    return tree, film


def test_single_rank_communicator_is_identity(pg):
    sc = pg.scenes.cornell(64, 64)
    t0, f0 = _train(pg, sc, False)
    t1, f1 = _train(pg, sc, True)
    assert np.array_equal(t0, t1)
    assert np.array_equal(f0[0], f1[0])
    t2, f2 = _train(pg, sc, True, mode="allgather")
    assert np.array_equal(t0, t2)
    assert np.array_equal(f0[0], f2[0])
    # the all-gather in many slices (pg_comm_allgather_records: rounds of PG_GATHER_SLICE records per rank
    # through one reused buffer, the last round padded): the same tree
    os.environ["PG_GATHER_SLICE"] = "777"
    try:
        t3, f3 = _train(pg, sc, True, mode="allgather")
    finally:
        del os.environ["PG_GATHER_SLICE"]
    assert np.array_equal(t0, t3)
    assert np.array_equal(f0[0], f3[0])


def test_record_allgather_equals_single_rank(pg):
    """The record all-gather exchange (pg_comm_allgather_records' arithmetic) emulated with
    two shard contexts on one GPU: every rank's records (pg_get_records) splatted into every rank's
    building tree in rank order (pg_splat_records) give the single-rank tree bit for bit, as
    test_tree_stats_allreduce_equals_single_rank does for the statistics all-reduce.  RCCL refuses two
    ranks on one device, so this is the multi-rank arithmetic of the library's all-gather path."""
    from mitsuba_path_guiding_amd.integrator import Device
    sc = pg.scenes.cornell(64, 48)
    cfg = dict(guiding=1, s_tree_threshold=300.0)
    full = Device(pg.capi.default_config(**cfg))
    full.upload(sc)
    parts = []
    for r in range(2):
        d = Device(pg.capi.default_config(rank=r, world_size=2, **cfg))
        d.upload(sc)
        parts.append(d)
    off = 0
    for it in range(4):
        full.render_pass(2 ** it, off, True)
        nfull = full.record_count()
        full.splat_local()
        full.refit(it)
        for d in parts:
            d.render_pass(2 ** it, off, True)
        recs = [d.get_records() for d in parts]
        assert sum(len(x) for x in recs) == 32 * nfull and all(len(x) for x in recs)
        for d in parts:
            for x in recs:  # rank order
                d.splat_records(x)
            d.refit(it)
        off += 2 ** it
    t = full.get_sdtree()
    assert all(np.array_equal(d.get_sdtree(), t) for d in parts)
    for d in parts + [full]:
        d.close()


def test_comm_calls_need_a_communicator(pg):
    from mitsuba_path_guiding_amd.integrator import Device, PGError
    d = Device(pg.capi.default_config())
    d.upload(pg.scenes.cornell(16, 16))
    with pytest.raises(PGError, match="no communicator"):
        d.comm_allreduce_tree_stats()
    with pytest.raises(PGError, match="no communicator"):
        d.comm_reduce_film(0)
    with pytest.raises(PGError, match="no communicator"):
        d.comm_allgather_records()
    d.close()
