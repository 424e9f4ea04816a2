"""GPU decompression (bzip2_amd/csrc/decomp.hip) against the reference.

Parity: the decoded bytes equal the original input, and for damaged streams the return code
equals what the reference build's BZ2_bzBuffToBuffDecompress (oracle/_ref, bzlib.c:1361-1410)
returns for the same bytes and output capacity.  The golden .bz2 files are the reference's own
(sample1..3) plus tests/golden/randomised.bz2 (made by tests/golden/make_randomised.py and
checked there against the reference)."""
import ctypes
import os
import random

import numpy as np
import pytest

import bzip2_amd as B
from tests import datagen, oracles as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def gold(name):
    with open(os.path.join(GOLD, name), "rb") as f:
        return f.read()


def compressed(data: bytes, level: int) -> bytes:
    return O.ref_compress(data, level) if O.has_ref() else O.orc_compress(data, level)


# ------------------------------------------------------------------ CPU: the table rule
@pytest.mark.skipif(not O.has_ref(), reason="reference build absent")
def test_decode_table_rule_is_kraft_equality():
    """decomp.hip accepts a table exactly when its code lengths satisfy Kraft with equality;
    the reference's BZ2_hbCreateDecodeTables (huffman.c:180-236) returns -1 otherwise."""
    L = O.ref()
    f = L.BZ2_hbCreateDecodeTables
    rng = random.Random(7)
    for _ in range(20000):
        eob = rng.randint(2, 257)
        if rng.random() < 0.5:
            lens = [1]
            while len(lens) < eob + 1:
                i = rng.randrange(len(lens))
                if lens[i] >= 20:
                    continue
                x = lens.pop(i)
                lens += [x + 1, x + 1]
            rng.shuffle(lens)
            if rng.random() < 0.5:
                j = rng.randrange(len(lens))
                lens[j] = max(1, min(20, lens[j] + rng.choice([-1, 1])))
        else:
            lens = [rng.randint(1, rng.choice([3, 8, 9, 12, 20])) for _ in range(eob + 1)]
        ln = (ctypes.c_ubyte * 300)(*lens)
        limit, base, perm = (ctypes.c_int * 30)(), (ctypes.c_int * 30)(), (ctypes.c_short * 600)()
        ok = f(limit, base, perm, ln, eob) >= 0
        assert ok == (sum(1 << (20 - x) for x in lens) == 1 << 20), lens


# ------------------------------------------------------------------ GPU
gpu = pytest.mark.gpu


def gpu_decode(stream: bytes, cap: int):
    return B.decompress_host(stream, cap)


@gpu
@pytest.mark.parametrize("i", [1, 2, 3])
def test_golden_samples(i):
    plain = gold(f"sample{i}.ref")
    rc, out = gpu_decode(gold(f"sample{i}.bz2"), len(plain) + 100)
    assert rc == 0 and out == plain
    # through the drop-in entry point
    assert B.buff_to_buff_decompress(gold(f"sample{i}.bz2"), len(plain)) == plain


@gpu
def test_randomised_block():
    rc, out = gpu_decode(gold("randomised.bz2"), 70000)
    assert rc == 0 and out == gold("randomised.out")


@gpu
@pytest.mark.parametrize("level", [1, 2, 5, 9])
def test_levels_mixed_content(level):
    data = (datagen.text(700_000, 11) + datagen.random_bytes(300_000, 3) + b"\x00" * 200_000 +
            bytes(range(256)) * 500 + b"ab" * 50_000 + datagen.text(100_000, 12))
    rc, out = gpu_decode(compressed(data, level), len(data))
    assert rc == 0 and out == data


@gpu
@pytest.mark.parametrize("data", [b"", b"a", b"aa", b"aaaa", b"aaaaa", b"a" * 259, b"a" * 260, b"ab",
                                  b"abcabcabc", b"\xff" * 1000, bytes(range(256))])
def test_edge_streams(data):
    s = compressed(data, 9)
    rc, out = gpu_decode(s, len(data) + 10)
    assert rc == 0 and out == data


@gpu
def test_periodic_and_single_byte_blocks():
    """Walk cycles shorter than the block (w^k blocks) and long runs (count bytes)."""
    for data, level in [(b"a" * 3_000_000, 9), (b"ab" * 500_000, 1), (b"hello" * 300_000, 2),
                        (b"abcabcabd" * 60_000, 9), (bytes([0xFB]) * 46_000_000, 9)]:
        rc, out = gpu_decode(compressed(data, level), len(data))
        assert rc == 0 and out == data, (data[:12], level)


@gpu
def test_many_blocks_round_trip_own_streams():
    """Streams of this library's compressor, -1 (many blocks) and -9."""
    data = datagen.text(30_000_000, 5) + datagen.random_bytes(2_000_000, 9)
    for level in (1, 9):
        s = B.buff_to_buff_compress(data, level)
        rc, out = gpu_decode(s, len(data))
        assert rc == 0 and out == data
        st = B.last_decode_stats()
        assert st["blocks"] >= len(data) // (100_000 * level)


@gpu
def test_output_capacity():
    data = datagen.text(1_000_000, 21)
    s = compressed(data, 1)
    for cap in (len(data), len(data) - 1, 0, 150_000, len(data) + 1):
        rc, out = gpu_decode(s, cap)
        want_rc, _ = O.ref_decompress(s, cap)
        assert rc == want_rc, cap
        if rc == 0:
            assert out == data


def damaged_cases(s: bytes, rng: random.Random, nflip: int, ntrunc: int):
    for _ in range(nflip):
        b = bytearray(s)
        pos = rng.randrange(len(b))
        b[pos] ^= 1 << rng.randrange(8)
        yield bytes(b)
    for _ in range(ntrunc):
        yield s[: rng.randrange(len(s))]
    for _ in range(ntrunc):  # a flip and a cut a few bytes after it
        b = bytearray(s)
        pos = rng.randrange(len(b) - 8)
        b[pos] ^= 1 << rng.randrange(8)
        yield bytes(b[: pos + rng.randint(1, 6)])
    # the first block's origPtr (stream bits 113..136) out of range, cut inside the next 16
    # bits: the reference reports the origPtr (decompress.c:348-351) before it needs them
    for cut in (17, 18, 19):
        b = bytearray(s)
        b[14] |= 0x40
        yield bytes(b[:cut])
    yield s[:3]
    yield b"BZh0" + s[4:]
    yield b"BZx9"
    yield s + b"trailing garbage"


@gpu
@pytest.mark.skipif(not O.has_ref(), reason="reference build absent")
def test_damaged_streams_match_reference_codes():
    rng = random.Random(0xBADC0DE)
    data = datagen.text(400_000, 31) + b"z" * 5000 + datagen.random_bytes(60_000, 4)
    s = compressed(data, 1)
    mism = []
    for d in damaged_cases(s, rng, 300, 40):
        rc, out = gpu_decode(d, len(data) + 1000)
        want_rc, want = O.ref_decompress(d, len(data) + 1000)
        if rc != want_rc or (rc == 0 and out != want):
            mism.append((rc, want_rc))
    assert not mism, mism[:10]


@gpu
def test_device_api_large_text():
    """Device-resident round trip at bench scale (size-independent property)."""
    import torch

    data = datagen.text(200_000_000, 77)
    s = B.buff_to_buff_compress(data, 9)
    d_in = torch.frombuffer(bytearray(s), dtype=torch.uint8).to("cuda:0")
    d_out = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda:0")
    rc, n = B.decompress_device(d_in.data_ptr(), len(s), d_out.data_ptr(), len(data) + 64,
                                stream_ptr=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert rc == 0 and n == len(data)
    assert d_out[:n].cpu().numpy().tobytes() == data
