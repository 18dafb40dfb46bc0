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


class Watchdog:
    """Host-side deadlines for the multi-rank start-up (what the reference's RemoteWorker handshake and
    StreamBackend error messages, sched_remote.h:50-236, give an operator: which worker is stuck where).

    Each rank reports every stage it enters on stderr ("[bench rank r/W dev d] stage ..."), with the time
    the previous one took, and -- once the process group is up -- in the group's key-value store.  A stage
    that outlives its deadline ends the rank with exit status 3, after naming, from the store, every rank
    whose last reported stage is not done (the stuck ranks); torch.distributed.run then stops the others.
    No exec and no GPU call: a plain thread and os._exit."""

    def __init__(self, rank, world, device=None, seconds=300.0, stream=None):
        import sys
        import threading
        import time
        self.rank, self.world, self.device = rank, world, device
        self.seconds = float(seconds)
        self.stream = stream or sys.stderr
        self.store = None
        self._lock = threading.Lock()
        self._stage, self._t0, self._limit, self._n, self._coll = None, time.monotonic(), None, 0, False
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._watch, daemon=True)
        self._thread.start()

    def _say(self, msg):
        self.stream.write(f"[bench rank {self.rank}/{self.world} dev {self.device}] {msg}\n")
        self.stream.flush()

    def attach_store(self):
        """The process group's store (after init_process_group): stages become visible to every rank."""
        try:
            import torch.distributed as dist
            self.store = dist.distributed_c10d._get_default_store()
        except Exception:  # noqa: BLE001 -- diagnostics only
            self.store = None
        self._publish()

    def _publish(self):
        if self.store is not None and self._stage is not None:
            try:
                self.store.set(f"pg_bench_stage_{self.rank}", f"{self._n}:{int(self._coll)}:{self._stage}")
            except Exception:  # noqa: BLE001
                pass

    def stage(self, name, seconds=None, collective=False):
        """Enter stage `name` (`collective`: the rank waits there for the others, so a deadline in it blames
        the ranks that are not in a collective)."""
        import time
        with self._lock:
            now = time.monotonic()
            if self._stage is not None:
                self._say(f"{self._stage}: done in {now - self._t0:.2f} s")
            self._stage, self._t0, self._coll = name, now, collective
            self._n += 1
            self._limit = self.seconds if seconds is None else float(seconds)
        self._say(f"stage {name} (deadline {self._limit:.0f} s)")
        self._publish()

    def done(self):
        self.stage("done", seconds=float("inf"), collective=True)
        self._stop.set()

    def others(self):
        """{rank: (stage number, in a collective, last reported stage)} of the ranks (empty without a store)."""
        out = {}
        if self.store is None:
            return out
        import datetime
        try:
            self.store.set_timeout(datetime.timedelta(seconds=2))
        except Exception:  # noqa: BLE001
            pass
        for r in range(self.world):
            try:
                n, coll, name = self.store.get(f"pg_bench_stage_{r}").decode().split(":", 2)
                out[r] = (int(n), coll == "1", name)
            except Exception:  # noqa: BLE001 -- a rank that never reported
                out[r] = (0, False, "(no report: never joined the store)")
        return out

    def report(self):
        """'stuck: ...; waiting: ...': ranks outside any collective are the stuck ones (the others wait for them);
        if every unfinished rank is inside a collective, those in the earliest stage."""
        ranks = {r: v for r, v in self.others().items() if v[2] != "done"}
        if not ranks:
            return "unknown (no store)"
        out_of_coll = {r for r, v in ranks.items() if not v[1]}
        if out_of_coll:
            stuck_set = out_of_coll
        else:
            first = min(v[0] for v in ranks.values())
            stuck_set = {r for r, v in ranks.items() if v[0] == first}
        stuck = ", ".join(f"rank {r} in {v[2]!r}" for r, v in sorted(ranks.items()) if r in stuck_set)
        wait = ", ".join(f"rank {r} in {v[2]!r}" for r, v in sorted(ranks.items()) if r not in stuck_set)
        return f"stuck: {stuck}" + (f"; waiting: {wait}" if wait else "")

    def _watch(self):
        import os
        import time
        while not self._stop.wait(0.25):
            with self._lock:
                stage, t0, limit = self._stage, self._t0, self._limit
            if stage is None or limit is None or time.monotonic() - t0 <= limit:
                continue
            self._say(f"DEADLINE: in stage {stage!r} for more than {limit:.0f} s; {self.report()}")
            os._exit(3)
