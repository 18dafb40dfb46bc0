"""Multi-GPU plumbing: one process per GPU, torch.distributed over RCCL (backend "nccl") on MI355X,
gloo on CPU for tests.  Replaces the reference's master/worker TCP/SSH scheduler
(include/mitsuba/core/sched_remote.h:50-236) for the ONE data-parallel hot path:

  * image tiles are sharded statically across ranks inside the C-ABI context (pg_config.rank /
    world_size, 32x32 tiles dealt round-robin; the RNG is keyed by the global pixel, so results do
    not depend on the number of ranks);
  * before each SD-tree refit (postprogression) every rank splats its own training records into
    its building tree, then the building-tree statistics (u64 fixed-point quadrant sums + record
    counts, pg_get_tree_stats) are all-reduced (SUM) and put back.  Integer sums are exact, so
    every rank refits a bit-identical tree, equal to splatting all records on one GPU
    (a few MB per iteration instead of all-gathering ~1 GB of records, and the
    splat work is split across ranks).  The record all-gather is kept as mode="allgather";
  * at the end the film tiles are sum-reduced to rank 0 (tiles are disjoint, so the sum is a gather).

The exchange takes any object with the Device interface it uses (splat_local / tree_stats_words /
get_tree_stats / put_tree_stats / record_count, or get_records / splat_records for "allgather"),
which lets the gloo tests run it against a CPU stand-in.
"""
import os

import numpy as np

RECORD_BYTES = 32


def env_rank():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def init(backend=None):
    """Initialise the default process group from the torchrun environment (127.0.0.1 rendezvous)."""
    import torch
    import torch.distributed as dist
    rank, world, local = env_rank()
    if world <= 1 or dist.is_initialized():
        return rank, world, local
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29512")
    if backend == "nccl":
        torch.cuda.set_device(local)
    dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


def make_exchange(on_device, mode="allreduce"):
    """Returns exchange(dev) for the postprogression slot; it returns every rank's record count.

    mode="allreduce": splat local records, all-reduce the building-tree statistics.
    mode="allgather": all-gather every rank's records and splat all of them into dev.
    on_device=True: buffers move device->device (RCCL over xGMI); False: through host memory (gloo).
    """
    import torch
    import torch.distributed as dist
    if mode not in ("allreduce", "allgather"):
        raise ValueError(f"unknown exchange mode {mode!r}")

    def exchange_allreduce(dev):
        world = dist.get_world_size()
        tdev = torch.device("cuda", torch.cuda.current_device()) if on_device else torch.device("cpu")
        counts = torch.zeros(world, dtype=torch.int64, device=tdev)
        dist.all_gather_into_tensor(counts, torch.tensor([int(dev.record_count())], dtype=torch.int64, device=tdev))
        dev.splat_local()
        words = int(dev.tree_stats_words())
        if on_device:
            t = torch.empty(words, dtype=torch.int64, device=tdev)
            dev.get_tree_stats(dst_ptr=t.data_ptr(), words=words)  # synchronous on the library's stream
            dist.all_reduce(t)
            torch.cuda.synchronize()
            dev.put_tree_stats(device_ptr=t.data_ptr(), words=words)
        else:
            t = torch.from_numpy(np.ascontiguousarray(dev.get_tree_stats()).view(np.int64).copy())
            dist.all_reduce(t)
            dev.put_tree_stats(t.numpy().view(np.uint64))
        return counts.cpu().tolist()

    def exchange(dev):
        world = dist.get_world_size()
        n_local = int(dev.record_count())
        tdev = torch.device("cuda", torch.cuda.current_device()) if on_device else torch.device("cpu")
        counts = torch.zeros(world, dtype=torch.int64, device=tdev)
        mine = torch.tensor([n_local], dtype=torch.int64, device=tdev)
        dist.all_gather_into_tensor(counts, mine)
        counts = counts.cpu().tolist()
        maxn = max(counts)
        if maxn == 0:
            return counts
        if on_device:
            buf = torch.empty(maxn * RECORD_BYTES, dtype=torch.uint8, device=tdev)
            torch.cuda.synchronize()
            dev.get_records(dst_ptr=buf.data_ptr(), max_records=n_local)
            gathered = torch.empty(world * maxn * RECORD_BYTES, dtype=torch.uint8, device=tdev)
            dist.all_gather_into_tensor(gathered, buf)
            torch.cuda.synchronize()
            base = gathered.data_ptr()
            for r in range(world):
                if counts[r]:
                    dev.splat_records(device_ptr=base + r * maxn * RECORD_BYTES, count=counts[r])
        else:
            host = np.zeros(maxn * RECORD_BYTES, np.uint8)
            local = dev.get_records()
            host[: len(local)] = local
            buf = torch.from_numpy(host)
            gathered = torch.empty(world * maxn * RECORD_BYTES, dtype=torch.uint8)
            dist.all_gather_into_tensor(gathered, buf)
            g = gathered.numpy()
            for r in range(world):
                if counts[r]:
                    off = r * maxn * RECORD_BYTES
                    dev.splat_records(g[off: off + counts[r] * RECORD_BYTES])
        return counts

    return exchange_allreduce if mode == "allreduce" else exchange


def init_capi_comm(dev):
    """The library's own RCCL communicator (pg_comm_init), the multi-GPU path of the C++ adapter:
    rank 0 draws the unique id (pg_comm_unique_id), torch.distributed broadcasts its bytes."""
    import torch.distributed as dist
    obj = [bytes(dev.comm_unique_id().tobytes()) if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    dev.comm_init(np.frombuffer(obj[0], np.uint8))


def make_capi_exchange(mode="allreduce"):
    """exchange(dev) through the library's communicator (after init_capi_comm).  Returns every
    rank's record count.

    mode="allreduce": splat the local records, then pg_comm_allreduce_tree_stats (in-place RCCL
    all-reduce of the device building statistics).
    mode="allgather": pg_comm_allgather_records (RCCL all-gather of every rank's records, each rank
    splats all of them); the same tree bit for bit."""
    if mode not in ("allreduce", "allgather"):
        raise ValueError(f"unknown exchange mode {mode!r}")
    if mode == "allgather":
        return lambda dev: dev.comm_allgather_records()

    def exchange(dev):
        import torch.distributed as dist
        counts = np.zeros(dist.get_world_size(), np.float64)
        counts[dist.get_rank()] = dev.record_count()
        dev.splat_local()
        dev.comm_allreduce_tree_stats()
        return [int(x) for x in dev.comm_allreduce_f64(counts)]

    return exchange


def reduce_film(rgbw, sumsq, on_device):
    """Sum-reduce the (disjoint-tile) films of all ranks to rank 0; returns numpy arrays on rank 0."""
    import torch
    import torch.distributed as dist
    tdev = torch.device("cuda", torch.cuda.current_device()) if on_device else torch.device("cpu")
    t = torch.from_numpy(np.stack([rgbw, sumsq])).to(tdev)
    dist.reduce(t, dst=0)
    out = t.cpu().numpy()
    return out[0], out[1]


def make_reduce_sum(on_device):
    """callable(np.ndarray float64) -> its element-wise sum over ranks (all-reduce)."""
    import torch
    import torch.distributed as dist

    def reduce_sum(x):
        tdev = torch.device("cuda", torch.cuda.current_device()) if on_device else torch.device("cpu")
        t = torch.from_numpy(np.ascontiguousarray(x, np.float64)).to(tdev)
        dist.all_reduce(t)
        return t.cpu().numpy()

    return reduce_sum


def max_over_ranks(value, on_device):
    import torch
    import torch.distributed as dist
    tdev = torch.device("cuda", torch.cuda.current_device()) if on_device else torch.device("cpu")
    t = torch.tensor([float(value)], dtype=torch.float64, device=tdev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value, on_device):
    import torch
    import torch.distributed as dist
    tdev = torch.device("cuda", torch.cuda.current_device()) if on_device else torch.device("cpu")
    t = torch.tensor([float(value)], dtype=torch.float64, device=tdev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
