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
