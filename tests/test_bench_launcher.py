"""bench.py's multi-rank launcher (the driver runs `python bench.py --gpus N` without torchrun):
with N > 1 and no WORLD_SIZE it starts N ranks through torch.distributed.run on 127.0.0.1, each
rank checks world == N; under torchrun a mismatched --gpus fails.  --plumbing-check exercises the
real launcher and process group (gloo) without a GPU or the library's compute path."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(kw)
    return env


def test_gpus_n_launches_n_ranks():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--plumbing-check"], env=_env(), capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    r = json.loads(line)
    assert r["n_gpus"] == 2 and r["rank_sum"] == 1.0
    assert sorted(x["rank"] for x in r["ranks"]) == [0, 1]
    assert sorted(x["local_rank"] for x in r["ranks"]) == [0, 1]
    assert all(x["world"] == 2 for x in r["ranks"])
    assert len({x["pid"] for x in r["ranks"]}) == 2  # one process per rank


def test_mismatched_world_fails():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--plumbing-check"],
                         env=_env(RANK="0", WORLD_SIZE="2", LOCAL_RANK="0"), capture_output=True, text=True, timeout=120)
    assert out.returncode != 0
    assert "--gpus 3" in out.stderr


def test_cpu_share_is_stated():
    sys.path.insert(0, ROOT)
    import bench
    cores, src = bench.cpu_share()
    assert cores >= 1 and src["used"] in src or src["used"] == "os.cpu_count"
    if "affinity" in src:
        assert cores <= src["affinity"]
    old = os.environ.get("OMP_NUM_THREADS")
    os.environ["OMP_NUM_THREADS"] = "3"
    try:
        cores3, src3 = bench.cpu_share()
        assert cores3 == min(3, cores) and src3["OMP_NUM_THREADS"] == 3
    finally:
        if old is None:
            del os.environ["OMP_NUM_THREADS"]
        else:
            os.environ["OMP_NUM_THREADS"] = old


def test_plumbing_check_reports_every_rank():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--plumbing-check"], env=_env(), capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    for r in (0, 1):  # per rank: its stages, and the first collective's completion
        assert f"[bench rank {r}/2 dev cpu] stage first collective" in out.stderr
        assert f"[bench rank {r}/2 dev cpu] first collective complete" in out.stderr


def test_deadline_names_the_stuck_rank():
    """A rank that never reaches the first collective: the waiting rank's deadline ends the job with a non-zero
    status and names the stuck rank and its stage (distributed.Watchdog), within a few deadlines."""
    import time
    t0 = time.time()
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--plumbing-check"],
                         env=_env(PG_BENCH_STALL_RANK="1", PG_BENCH_DEADLINE="8"), capture_output=True, text=True,
                         timeout=300)
    assert out.returncode != 0
    assert "DEADLINE" in out.stderr, out.stderr[-3000:]
    assert "stuck: rank 1 in 'stall (test hook)'" in out.stderr, out.stderr[-3000:]
    assert time.time() - t0 < 120


def test_headline_frac_source():
    """The line's headline fraction uses the committed rocprof duration only for the profiled workload."""
    sys.path.insert(0, ROOT)
    import bench
    dom = {"avg_launch_ms_rocprof": 2.0}
    r = bench.headline_frac(2000.0, 4e9, 1.9, dom, profiled=True)
    assert r["avg_launch_ms"] == 2.0 and abs(r["achieved"] - 2000.0) < 1e-6 and r["frac"] == 0.25
    assert r["frac_hip_events"] == 0.25 and "box_difference" in r  # 1.9 vs 2.0 ms: 5 %
    r = bench.headline_frac(500.0, 1e8, 0.2, dom, profiled=False)
    assert r["avg_launch_ms"] == 0.2 and r["frac"] == round(500.0 / bench.HBM_PEAK_GBS, 5)
    assert "not this one" in r["frac_source"]
    assert bench.headline_frac(500.0, 1e8, 0.2, {}, profiled=True)["frac_source"] == "HIP events, this run"
