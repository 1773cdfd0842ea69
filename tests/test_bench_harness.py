"""CPU: the N > 1 bench harness (stream sharding, barrier-bracketed timing, max over ranks) with
world_size 2 over gloo — the same functions bench.py runs over RCCL on the GPU box."""
import os
import socket
import sys
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        S, steps = 3, 4
        seeds = bench.stream_seeds(1000, rank, S)
        every = [None] * world
        dist.all_gather_object(every, seeds)
        # rank 1 is deliberately slower: the job time must be the slowest rank's
        el = bench.timed_region(lambda: time.sleep(0.05 + 0.15 * rank), lambda: None, dist)
        job = bench.max_over_ranks(el, dist, "cpu")
        q.put((rank, every, el, job, bench.aggregate_rate(world, S, steps, job)))
    finally:
        dist.destroy_process_group()


def test_two_rank_harness_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seeds = res[0][1]
    flat = [x for r in seeds for x in r]
    assert len(set(flat)) == len(flat)            # disjoint stream shards
    assert seeds[1][0] == seeds[0][-1] + 1        # contiguous global stream numbering
    jobs = {r[3] for r in res}
    assert len(jobs) == 1                         # every rank reports the same (max) time
    job = jobs.pop()
    assert job >= max(r[2] for r in res) - 1e-9 and job >= 0.2
    assert res[0][4] == pytest.approx(world * 3 * 4 / job)


def test_bench_launches_n_ranks_dry_cpu():
    """`bench.py --gpus 2` starts two rank processes itself (no torchrun) and rank 0 reports
    n_gpus = 2 with disjoint, contiguous stream seeds (--dry-cpu: gloo, NumPy stand-in step)."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-cpu",
                        "--streams", "3", "--n", "32", "--steps", "3", "--warmup", "1",
                        "--preroll", "2"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout               # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["dry_run"]
    seeds = d["stream_seeds_by_rank"]
    assert seeds == [[1000, 1001, 1002], [1003, 1004, 1005]]
    assert d["value"] > 0


@pytest.mark.parametrize("tracker,streams", [("deepocsort", 1), ("hybridsort", 3)])
def test_bench_config_dry_cpu_two_ranks(tracker, streams):
    """`bench.py --gpus 2 --dry-cpu --tracker deepocsort|hybridsort`: the C4 / C5 harness (their
    streams with embeddings, sharded s mod G: rank r takes global streams r, r + G, ...), two
    rank processes over gloo, rank 0's single JSON line with the aggregate."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-cpu",
                        "--tracker", tracker, "--streams", str(streams), "--n", "24", "--dim", "16",
                        "--steps", "3", "--warmup", "1", "--seed", "2000"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["tracker"] == tracker and d["streams_per_gpu"] == streams
    seeds = d["stream_seeds_by_rank"]
    assert seeds == [[2000 + 2 * k for k in range(streams)], [2001 + 2 * k for k in range(streams)]]
    assert d["value"] > 0


def test_config_seeds_shard_mod_g():
    """C5's 64 streams over 8 ranks: rank r holds global streams r, r + 8, ... (8 each), every
    stream exactly once."""
    G, per = 8, 8
    every = [bench.config_seeds(0, r, G, per) for r in range(G)]
    flat = sorted(x for r in every for x in r)
    assert flat == list(range(G * per))
    assert all(all(x % G == r for x in every[r]) for r in range(G))


def test_bench_defaults_per_tracker():
    a = bench.parse([])
    assert (a.tracker, a.n, a.streams) == ("bytetrack", 1024, 2048)
    a = bench.parse(["--tracker", "deepocsort"])
    assert (a.n, a.streams) == (2048, 1)     # C4: 8 streams over 8 GPUs
    a = bench.parse(["--tracker", "hybridsort"])
    assert (a.n, a.streams) == (4096, 8)     # C5: 64 streams over 8 GPUs
