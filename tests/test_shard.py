"""One stream sharded across ranks (bzip2_amd/shard.py) on CPU: the block-cut chain
against the whole-stream cut rule, and end-to-end gloo runs (world size 2 and 3) whose rank-0
stream must equal the oracle's stream of the whole input, with the CPU stand-in backend
(tests/shard_cpu.py).  The GPU backend runs the same code in tests/test_gpu.py."""
import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bzip2_amd import shard as S
from tests import datagen, oracles as O
from tests.shard_cpu import CpuBackend, chunks, cuts_whole


def _inputs():
    rnd = random.Random(7)
    txt = datagen.text(260_000, 11)
    runs = bytearray()
    while len(runs) < 250_000:
        runs += bytes([rnd.choice(b"ab\x00\xff")]) * rnd.choice([1, 2, 3, 4, 5, 254, 255, 256, 509, 510, 511, 3000])
    return {
        "text": txt,
        "runs": bytes(runs),
        "text_run_text": txt[:90_000] + b"q" * 150_000 + txt[90_000:200_000],
        "one_byte": b"z" * 900_000,
        "tail_len1": b"k" * 25_000 * 4 + b"x",  # ends with a 1-byte chunk
        # the first run ends at the stream's last byte with the open block already full there
        # (-1: 19996 chunks of 255 fill 99,980 bytes; the last chunk brings it past nblockMAX)
        "full_then_last": b"a" * (255 * 19996 + 4) + b"b",
        "runs_of_4": b"aaaabbbb" * 60_000,  # RLE1 grows the input by 5/4
    }


@pytest.mark.parametrize("name", list(_inputs()))
def test_cut_rule_matches_oracle_blocks(name):
    data = _inputs()[name]
    for level in (1, 2):
        cuts = cuts_whole(data, level)
        st, ln, sz = chunks(np.frombuffer(data, np.uint8))
        bounds = [0] + cuts + [len(data)]
        sizes = [int(sz[(st >= a) & (st < b)].sum()) for a, b in zip(bounds, bounds[1:])]
        _, offs, _ = O.orc_rle1(data, level, 1)
        assert sizes == [b - a for a, b in zip(offs, offs[1:])]


def _chain_local(data, level, bounds_):
    """Step 1 of compress_sharded for every shard in one process (message passed locally)."""
    be = CpuBackend(level)
    msg, cuts = None, []
    n = len(data)
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    for r, (a, b) in enumerate(zip(bounds_, bounds_[1:])):
        c, msg = S.chain_piece(be, t[a:b], a, n, msg, final=(r == len(bounds_) - 2))
        cuts += c
    return cuts


@pytest.mark.parametrize("name", list(_inputs()))
def test_chain_cuts_equal_whole_stream_cuts(name):
    data = _inputs()[name]
    rnd = random.Random(len(data))
    n = len(data)
    for level in (1, 2):
        want = cuts_whole(data, level)
        for trial in range(6):
            k = rnd.choice([2, 3, 5, 9])
            inner = sorted(rnd.sample(range(1, n), k - 1))
            if trial == 0:  # boundaries right at and around cuts
                inner = sorted({max(1, min(n - 1, c + d)) for c in want[:3] for d in (-1, 0, 1)})
            if trial == 1:
                inner = [n - 1]  # a 1-byte last shard
            bnd = [0] + inner + [n]
            assert _chain_local(data, level, bnd) == want, (level, bnd)


def test_extend_run_arithmetic_matches_chunk_walk():
    for L in (1, 255, 256, 100_000, 3_000_000):
        for fill in (0, 5, 99_000):
            data = b"r" * L + b"s"
            st, ln, sz = chunks(np.frombuffer(data, np.uint8))
            mx = S.nblock_max(1)
            want, s = [], -fill
            outpos = np.concatenate([[0], np.cumsum(sz)[:-1]])
            for i in range(len(st)):
                if outpos[i] - s >= mx and st[i] != len(data) - 1:
                    want.append(int(st[i]))
                    s = int(outpos[i])
            got = []
            t, f = S.extend_run(0, fill, L, mx, got, len(data) - 1)
            assert got == [c for c in want if c < L]
            assert t == int(st[-2]) and f == int(outpos[-2] - s) if L > 0 else True


def test_shift_bits():
    rnd = random.Random(3)
    for _ in range(50):
        nb = rnd.randint(1, 60)
        raw = bytes(rnd.randrange(256) for _ in range((nb + 7) // 8))
        sh = rnd.randrange(8)
        bits = np.unpackbits(np.frombuffer(raw, np.uint8))[:nb]
        want = np.packbits(np.concatenate([np.zeros(sh, np.uint8), bits]))
        got = S.shift_bits(torch.tensor(list(raw), dtype=torch.uint8), nb, sh).numpy()
        assert got.tolist() == want.tolist()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, cases, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        for key, (data, level, bnd) in cases.items():
            t = torch.frombuffer(bytearray(data[bnd[rank]:bnd[rank + 1]]), dtype=torch.uint8)
            res = S.compress_sharded(t, bnd[rank], len(data), level, backend=CpuBackend(level))
            if rank == 0:
                out[key] = res.numpy().tobytes()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_stream_equals_whole_stream(world):
    inp = _inputs()
    rnd = random.Random(world)
    cases = {}
    for name, data in inp.items():
        n = len(data)
        for level in (1, 3):
            bnd = [0] + sorted(rnd.sample(range(1, n), world - 1)) + [n]
            cases[(name, level, "rand")] = (data, level, bnd)
    # a shard that owns no block start, and shards that split the long run
    d = inp["text_run_text"]
    cases[("nostart", 1, "x")] = (d, 1, [0] + [100_000 + 1000 * i for i in range(1, world)] + [len(d)])
    cases[("tiny", 2, "x")] = (inp["text"][:5000], 2, [0] + list(range(1, world)) + [5000])
    port = _free_port()
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, port, cases, out), nprocs=world, join=True)
    for key, (data, level, bnd) in cases.items():
        assert out[key] == O.orc_compress(data, level), (key, bnd)


def test_single_process_without_process_group():
    data = _inputs()["runs"]
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    res = S.compress_sharded(t, 0, len(data), 2, backend=CpuBackend(2))
    assert res.numpy().tobytes() == O.orc_compress(data, 2)
