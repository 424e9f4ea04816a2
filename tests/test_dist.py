"""Multi-rank logic of bench.py on CPU (gloo, world size 2): every rank reports the slowest
rank's time, the job value counts every rank's bytes, and ranks hold distinct inputs (their
shards of one stream in `--mode stream`, the default for N > 1, or independent streams in
`--mode independent`).  The sharded stream itself is tested in test_shard.py."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from tests import datagen


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        elapsed = 1.0 + rank  # rank 1 is the slow one
        t = bench.max_over_ranks(elapsed, "cpu")
        v = bench.job_mbps(1000, world, 3, t)
        out[rank] = (t, v)
    finally:
        dist.destroy_process_group()


def test_two_ranks_max_time_and_job_value():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    for r in range(world):
        t, v = out[r]
        assert t == 2.0
        assert v == pytest.approx(1000 * world * 3 / 2.0 / 1e6)


def test_ranks_get_distinct_objects():
    a = datagen.text(100_000, bench.rank_seed(0))
    b = datagen.text(100_000, bench.rank_seed(1))
    assert len(a) == len(b) == 100_000 and a != b


def _run_bench(args, env_extra):
    import json
    import subprocess
    import sys

    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=240)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    return r.returncode, lines, r.stderr


def test_bench_gpus_n_launches_n_ranks():
    """`bench.py --gpus 2` with no outside launcher starts 2 ranks (torch.distributed.run on
    127.0.0.1); the probe mode stops each rank before any GPU call."""
    rc, lines, err = _run_bench(["--gpus", "2"], {"BZG_BENCH_PROBE": "1", "BZG_DIST_BACKEND": "gloo"})
    assert rc == 0, err[-2000:]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert all(x["world"] == 2 and x["master"] == "127.0.0.1" for x in lines)
    assert sorted(x["local_rank"] for x in lines) == [0, 1]


def test_bench_world_size_must_match_gpus():
    rc, lines, err = _run_bench(["--gpus", "2"], {"BZG_BENCH_PROBE": "1", "WORLD_SIZE": "3", "RANK": "0"})
    assert rc == 2 and not lines and "!= --gpus 2" in err
    rc, lines, _ = _run_bench(["--gpus", "1"], {"BZG_BENCH_PROBE": "1"})
    assert rc == 0 and lines == [{"rank": 0, "world": 1, "local_rank": 0, "master": None}]


def test_bench_total_bytes_strong_layout():
    """`--total-bytes T` (BASELINE config 3, strong scaling): ONE stream of T bytes, rank r holding
    input[T r / N, T (r + 1) / N); the shards tile [0, T) in rank order."""
    T = 1_000_000_007
    for world in (2, 3):
        rc, lines, err = _run_bench(["--gpus", str(world), "--total-bytes", str(T)],
                                    {"BZG_BENCH_PROBE": "1", "BZG_DIST_BACKEND": "gloo"})
        assert rc == 0, err[-2000:]
        lines.sort(key=lambda x: x["rank"])
        assert [x["rank"] for x in lines] == list(range(world))
        assert all(x["scaling"] == "strong" and x["mode"] == "stream" and x["job_bytes"] == T for x in lines)
        assert lines[0]["lo"] == 0 and lines[-1]["lo"] + lines[-1]["n"] == T
        assert all(lines[r]["lo"] + lines[r]["n"] == lines[r + 1]["lo"] for r in range(world - 1))
        assert max(x["n"] for x in lines) - min(x["n"] for x in lines) <= 1


def test_job_layout_weak_and_strong():
    import argparse

    a = argparse.Namespace(total_bytes=0, bytes=1000, mode=None)
    assert bench.job_layout(a, 1, 0)["mode"] == "independent"
    w = bench.job_layout(a, 4, 2)
    assert (w["scaling"], w["mode"], w["lo"], w["n"], w["job_bytes"]) == ("weak", "stream", 2000, 1000, 4000)
    a.total_bytes = 10
    s = [bench.job_layout(a, 3, r) for r in range(3)]
    assert [(x["lo"], x["n"]) for x in s] == [(0, 3), (3, 3), (6, 4)]
    assert all(x["scaling"] == "strong" and x["seed"] == bench.rank_seed(0) for x in s)
