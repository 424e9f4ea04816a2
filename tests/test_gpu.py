"""GPU parity tests: every stage of the HIP path (through the C ABI) against the oracle on the
same seeded inputs, whole streams against the reference's golden vectors and against the
reference build (oracle/_ref), and size-independent properties at larger sizes."""
import bz2
import ctypes
import os
import random

import numpy as np
import pytest

import bzip2_amd as B
from tests import datagen, oracles as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def gold(name):
    with open(os.path.join(GOLD, name), "rb") as f:
        return f.read()


def expected(data: bytes, level: int) -> bytes:
    """The reference's output: the reference build when present, else the oracle (same
    output on every input the tests use, pinned in test_oracle.py)."""
    if O.has_ref():
        return O.ref_compress(data, level)
    return O.orc_compress(data, level)


# ------------------------------------------------------------------ stage parity
def gpu_rle1(data: bytes, level: int, tail_merge: int = 1):
    L = B.lib()
    cap = len(data) + len(data) // 4 + 64
    blocks = ctypes.create_string_buffer(cap)
    maxb = len(data) // 90000 + 8
    offs = (ctypes.c_uint32 * (maxb + 1))()
    crcs = (ctypes.c_uint32 * maxb)()
    nb = ctypes.c_uint32(0)
    rc = L.bzg_stage_rle1(data, len(data), level, tail_merge, blocks, cap, offs, crcs, ctypes.byref(nb), maxb)
    assert rc == 0, rc
    o = [offs[i] for i in range(nb.value + 1)] if nb.value else [0]
    return blocks.raw[: o[-1]], o, [crcs[i] for i in range(nb.value)]


def gpu_bwt(blocks: bytes, offs):
    nb = len(offs) - 1
    out = ctypes.create_string_buffer(max(len(blocks), 1))
    orig = (ctypes.c_int32 * max(nb, 1))()
    o32 = (ctypes.c_uint32 * (nb + 1))(*offs)
    rc = B.lib().bzg_stage_bwt(blocks, o32, nb, out, orig)
    assert rc == 0, rc
    return out.raw[: len(blocks)], [orig[i] for i in range(nb)]


def gpu_mtf(bwt: bytes, offs):
    nb = len(offs) - 1
    total = offs[-1]
    cap = total + 8 * nb + 16
    mtfv = (ctypes.c_uint16 * cap)()
    moff = (ctypes.c_uint32 * (nb + 1))()
    nmtf = (ctypes.c_uint32 * nb)()
    freq = (ctypes.c_uint32 * (nb * 258))()
    o32 = (ctypes.c_uint32 * (nb + 1))(*offs)
    rc = B.lib().bzg_stage_mtf(bwt, o32, nb, mtfv, cap, moff, nmtf, freq)
    assert rc == 0, rc
    if nb and moff[nb] > 0:  # a short buffer is refused, not overrun
        assert B.lib().bzg_stage_mtf(bwt, o32, nb, mtfv, moff[nb] - 1, moff, nmtf, freq) == B.BZ_OUTBUFF_FULL
    arr = np.frombuffer(mtfv, dtype=np.uint16)
    fr = np.frombuffer(freq, dtype=np.uint32).reshape(nb, 258)
    return [arr[moff[b]: moff[b] + nmtf[b]].copy() for b in range(nb)], fr


def _huffman_tables(seed, n):
    rng = random.Random(seed)
    out = [[10] * 6, [int(2 ** (i // 2)) if i < 40 else 1 for i in range(258)]]
    fib = [1, 1]
    while len(fib) < 60:
        fib.append(fib[-1] + fib[-2])
    out.append(fib[:28])  # depth 27 > 17: rescale rounds (sum 832,039 <= nMTF max, weights fit int32)
    while len(out) < n:
        alpha = rng.randint(3, 258)
        mode = rng.random()
        if mode < 0.3:
            f = [rng.randint(0, 5) for _ in range(alpha)]
        elif mode < 0.6:
            f = [int(rng.paretovariate(1.1) * 10) for _ in range(alpha)]
        else:
            f = [rng.randint(0, 900_000 // alpha) for _ in range(alpha)]
        out.append(f)
    return out


@pytest.mark.parametrize("spec_max", ["512", "0"])
def test_code_lengths_vs_reference(spec_max, monkeypatch):
    """A8 (huffman.c:63-148) on the GPU: tie order, rescale rounds, random tables; rounds 1 and 2
    tried at once (k_huff_spec, forced on for the 400 tables) and one after another
    (BZG_HUFF_SPEC_MAX=0)."""
    if spec_max is not None:
        monkeypatch.setenv("BZG_HUFF_SPEC_MAX", spec_max)
    tables = _huffman_tables(11, 400)
    got = B.code_lengths(tables)
    for f, g in zip(tables, got):
        want = O.ref_code_lengths(f) if O.has_ref() else O.orc_code_lengths(f)
        assert g == want, (len(f), f[:8])
    assert got[0] == [3, 3, 2, 3, 2, 3]
    assert max(got[1]) == 17 and max(got[2]) <= 17  # table 2 needed rescale rounds (depth 27 unscaled)


def test_huff_spec_stream_equals_serial(monkeypatch):
    """k_huff_spec in a whole stream: the first 20 MB of the bench text (seed of bench.py's rank
    0) has 5 of its 552 table runs needing a second Huffman round (blocks 6, 15, 17: iterations
    0-3).  Rounds 1 and 2 at once (forced on every launch) and one after another give the same
    stream, the reference's."""
    data = datagen.text(20_000_000, 0x5EED0001)
    monkeypatch.setenv("BZG_HUFF_SPEC_MAX", "100000")
    spec = B.buff_to_buff_compress(data, 9)
    monkeypatch.setenv("BZG_HUFF_SPEC_MAX", "0")
    serial = B.buff_to_buff_compress(data, 9)
    assert spec == serial
    assert spec == expected(data, 9)


RLE_CASES = {
    "text": lambda: datagen.text(2_500_000, 21),
    "random": lambda: datagen.random_bytes(700_000, 22),
    "single": lambda: datagen.single_byte(3_000_000, 0x61),
    "runs": lambda: bytes(np.repeat(np.frombuffer(datagen.random_bytes(40_000, 23), np.uint8) % 7,
                                    np.random.default_rng(5).integers(1, 700, 40_000)).tobytes()[:2_000_000]),
}


@pytest.mark.parametrize("case", list(RLE_CASES))
@pytest.mark.parametrize("level", [1, 9])
def test_rle1_segmentation_crc(case, level):
    data = RLE_CASES[case]()
    for tm in (1, 0):
        assert gpu_rle1(data, level, tm) == O.orc_rle1(data, level, tm), (case, level, tm)


def test_rle1_edge_inputs():
    for data in [b"", b"a", b"ab", b"aaaa", b"aaaaa", b"a" * 255, b"a" * 256, b"a" * 259, b"ab" * 3]:
        assert gpu_rle1(data, 1) == O.orc_rle1(data, 1), data[:10]
    edge = bytes((i * 7 + (i >> 8)) % 251 + 1 for i in range(99_982))
    for tm in (0, 1):
        assert gpu_rle1(edge, 1, tm) == O.orc_rle1(edge, 1, tm)


def _blocks_of(data, level):
    blocks, offs, _ = O.orc_rle1(data, level)
    return blocks, offs


@pytest.mark.parametrize("case", ["text", "random", "small_mixed", "low_alpha"])
def test_bwt_matches_oracle(case):
    rng = random.Random(3)
    if case == "text":
        blocks, offs = _blocks_of(datagen.text(2_000_000, 31), 9)
    elif case == "random":
        blocks, offs = _blocks_of(datagen.random_bytes(900_000, 32), 3)
    elif case == "low_alpha":
        blocks, offs = _blocks_of(bytes(rng.randrange(2) for _ in range(300_000)), 1)
    else:
        parts = []
        for n in [1, 2, 3, 5, 17, 64, 100, 1000, 2047, 2048, 2049, 4097, 9000]:
            alpha = rng.choice([2, 3, 26, 256])
            p = bytes(rng.randrange(alpha) for _ in range(n))
            parts.append(p)
        offs = [0]
        for p in parts:
            offs.append(offs[-1] + len(p))
        blocks = b"".join(parts)
    bwt, orig = gpu_bwt(blocks, offs)
    for b in range(len(offs) - 1):
        blk = blocks[offs[b]:offs[b + 1]]
        L, o, per = O.orc_bwt(blk)
        if per != len(blk) and per > 1:
            continue  # periodic root: A5 resolver is tested separately
        assert bwt[offs[b]:offs[b + 1]] == L, (case, b, len(blk))
        assert orig[b] == o, (case, b, len(blk))


def _periodic_blocks(seed):
    """Exactly periodic blocks w^k of every A5 regime: one B* per period (device closed form;
    single-byte runs after RLE1, k around the 1024-item radix block and the 8-item limits),
    several B* per period (host model: short and long roots, dense small alphabets, text)."""
    rng = random.Random(seed)
    parts = []
    for c in (0x00, 0x61, 0xFB, 0xFF):
        parts.append(bytes([c] * 4 + [0xFB]) * rng.choice([2, 9, 1025, 1026, 1027, 19997, 179997]))
    for w, k in ((b"ab", 4096), (b"abc", 17), (b"abc", 1026), (b"aab", 300), (b"abcabcabd", 11109),
                 (b"bababac", 4096)):
        parts.append(w * k)
    # several B* per period in pairwise different buckets (device closed form, k_copyrank_cf)
    for w, k in ((b"hello world\n", 9), (b"hello world\n", 1025), (b"abac", 2), (b"abac", 1026),
                 (b"cab", 1025), (b"abac", 224_995)):
        parts.append(w * k)
    for _ in range(40):
        mode = rng.random()
        if mode < 0.4:
            w = bytes(rng.randrange(rng.choice([2, 3, 4, 256])) for _ in range(rng.randint(2, 12)))
        elif mode < 0.7:
            w = bytes(rng.randrange(rng.choice([2, 3])) for _ in range(rng.randint(8, 300)))
        else:
            w = datagen.text(rng.randint(20, 3000), rng.randrange(1000))
        k = rng.randint(2, max(2, min(60_000, 900_000 // len(w))))
        if len(set(w)) > 1:
            parts.append(w * k)
    offs = [0]
    for p_ in parts:
        offs.append(offs[-1] + len(p_))
    return b"".join(parts), offs


def test_periodic_blocks_origptr_vs_reference():
    """A5 on the device (origptr.hip) and the host copy-rank model (copyrank.cpp) through the
    stage ABI: every periodic block's origPtr and last column against the reference build."""
    if not O.has_ref():
        pytest.skip("needs oracle/_ref")
    blocks, offs = _periodic_blocks(42)
    bwt, orig = gpu_bwt(blocks, offs)
    for b in range(len(offs) - 1):
        blk = blocks[offs[b]:offs[b + 1]]
        want_l, want_o = O.ref_blocksort(blk)
        assert orig[b] == want_o, (b, blk[:16], len(blk))
        assert bwt[offs[b]:offs[b + 1]] == want_l, (b, len(blk))


def test_periodic_roots_resolved_on_device():
    """periodic roots with several B* offsets in pairwise different buckets are
    resolved by the device (k_copyrank_cf): a stream of only such blocks leaves nothing to the
    host model; mixed with shared-bucket roots, only those reach it.  Bytes vs the reference."""
    if not O.has_ref():
        pytest.skip("needs oracle/_ref")
    # root lengths divide the -1 block (99,981 = 3^3 7 23^2): every block is exactly periodic;
    # q = 2..6 B* offsets per root
    roots = (b"cab", b"</text>", b"</revis", b"</revisio", b"></title>\n  <id></id>", b"></title>\n  <id></id>\n ",
             b"  <id></id>\n  <revision>\n  ")
    data = b"".join(w * (99_981 // len(w)) * 2 for w in roots)
    assert B.buff_to_buff_compress(data, 1) == O.ref_compress(data, 1)
    st = B.last_stats()
    # (RLE1 of the last root's runs of spaces shifts the later cuts: 8 blocks stay exactly periodic
    # with q >= 2, computed from the oracle's blocks in round 5)
    assert st["a5_roots"] == 8 and st["a5_host"] == 0, st
    mixed = b"abcabcabd" * (99_981 // 9) * 2 + data  # 2 more blocks, q = 3 in shared buckets: host model
    assert B.buff_to_buff_compress(mixed, 1) == O.ref_compress(mixed, 1)
    st = B.last_stats()
    assert st["a5_roots"] == 10 and st["a5_host"] == 2, st


def test_periodic_blocks_stream_vs_reference():
    """Whole streams made of exactly periodic blocks (|w| divides the -1 block size 99,981):
    several roots per stream, RLE1 single-byte blocks included."""
    if not O.has_ref():
        pytest.skip("needs oracle/_ref")
    rng = random.Random(7)
    segs = [bytes([0x61]) * 450_000]
    for ln in (3, 7, 9, 21, 23, 27, 63, 69, 161, 189, 207):
        w = bytes(rng.randrange(rng.choice([2, 3, 26])) for _ in range(ln))
        if len(set(w)) > 1:
            segs.append(w * (99_981 // ln) * 2)
    data = b"".join(segs)
    assert B.buff_to_buff_compress(data, 1) == O.ref_compress(data, 1)


def _long_repeat_blocks():
    """Aperiodic blocks with long repeats: deep string-tile groups (kDWave), deep S1 buckets
    (kDBig) and big radix-round groups all end in the doubling fallback."""
    rng = random.Random(11)
    w = bytes(rng.randrange(256) for _ in range(3000))
    parts = [
        w * 50 + b"x",                                   # 50-member groups, LCP up to 147k
        b"ab" * 40_000 + b"c",                           # two huge S1 buckets, LCP up to 80k
        (b"abcabcabd" * 9000)[:-1] + b"e",               # near-periodic, period 9
        bytes(rng.randrange(2) for _ in range(400)) * 200 + b"\x02",  # 200-member groups, binary
        datagen.text(20_000, 5) * 12 + b"!",             # text repeats, 12-member groups
        bytes(rng.randrange(4) for _ in range(70_000)),  # small alphabet, no long repeats
    ]
    offs = [0]
    for p_ in parts:
        offs.append(offs[-1] + len(p_))
    return b"".join(parts), offs


def test_bwt_long_repeats_fallback():
    blocks, offs = _long_repeat_blocks()
    bwt, orig = gpu_bwt(blocks, offs)
    for b in range(len(offs) - 1):
        blk = blocks[offs[b]:offs[b + 1]]
        L, o, per = O.orc_bwt(blk)
        assert per == len(blk), b  # all aperiodic
        assert bwt[offs[b]:offs[b + 1]] == L, b
        assert orig[b] == o, b


def _deep_pair_blocks():
    """Blocks whose deep tied groups are mostly pairs, for the S3 pair resolver (sort.hip
    k_pair_end / k_pair_long / k_pair_resolve): twice-copied passages (run ends compare a few
    characters), pairs whose run ends inside a three-copy group (a run-end scan past
    kPairShort, the k_pair_long path), self-overlapping copies (a pair's partner run crosses its
    own run), and copies that wrap round the block end (cyclic comparison)."""
    rng = random.Random(23)

    def rnd(k):
        return bytes(rng.randrange(256) for _ in range(k))

    out = []
    p = rnd(5000)  # twice-copied passage, random continuations
    out.append(rnd(3000) + p + rnd(2000) + p + rnd(4000))
    s = rnd(6000)  # "x"+S twice, "y"+S once: the x-pairs share 6001 chars, their successors are triples
    out.append(rnd(1000) + b"x" + s + rnd(500) + b"x" + s + rnd(700) + b"y" + s + rnd(900))
    u = rnd(6000)  # u u u[:3000]: pairs (i, i+6000) overlap themselves
    out.append(rnd(800) + u + u + u[:3000] + b"\x00" + rnd(1200))
    w = rnd(4000)  # one copy at the end, one at the start: comparisons wrap round
    out.append(w[2000:] + rnd(3000) + w + rnd(1500) + w[:2000])
    t = datagen.text(30_000, 77)  # text passage twice inside text
    out.append(datagen.text(50_000, 78) + t + datagen.text(20_000, 79) + t + datagen.text(10_000, 80))
    offs = [0]
    for p_ in out:
        offs.append(offs[-1] + len(p_))
    return b"".join(out), offs


def test_bwt_deep_pairs():
    blocks, offs = _deep_pair_blocks()
    bwt, orig = gpu_bwt(blocks, offs)
    for b in range(len(offs) - 1):
        blk = blocks[offs[b]:offs[b + 1]]
        L, o, per = O.orc_bwt(blk)
        assert per == len(blk), b
        assert bwt[offs[b]:offs[b + 1]] == L, b
        assert orig[b] == o, b


def test_deep_pairs_stream():
    blocks, _ = _deep_pair_blocks()
    assert B.buff_to_buff_compress(blocks, 9) == expected(blocks, 9)


def test_many_deep_groups_repeats():
    """Enwik-like long repeats at scale: 400 MB of text with a quarter overwritten by copies of
    earlier passages (2-200 kB) gives tens of millions of groups still tied after the string
    passes (more than one launch of one workgroup per group could hold): the doubling fallback
    must order every one of them (the whole stream against the reference)."""
    torch = pytest.importorskip("torch")
    import bench

    n = 400_000_000
    d = torch.frombuffer(bytearray(datagen.text(n, 0x5EED0007)), dtype=torch.uint8).to("cuda")
    bench.add_repeats(d, 0.25)
    data = d.cpu().numpy().tobytes()
    cap = B.bound(n)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    nb, _, _ = B.compress_device(d.data_ptr(), n, 9, out.data_ptr(), cap)
    torch.cuda.synchronize()
    got = out[:nb].cpu().numpy().tobytes()
    del d, out
    assert got == expected(data, 9)


def test_long_repeats_streams():
    blocks, _ = _long_repeat_blocks()
    for level in (1, 9):
        assert B.buff_to_buff_compress(blocks, level) == expected(blocks, level)


def test_bwt_single_symbol_blocks():
    blocks = b"a" * 5000 + b"\xfb" * 3 + b"z"
    offs = [0, 5000, 5003, 5004]
    bwt, orig = gpu_bwt(blocks, offs)
    assert bwt == blocks and orig == [0, 0, 0]


@pytest.mark.parametrize("case", ["text", "random"])
def test_mtf_matches_oracle(case):
    data = datagen.text(1_500_000, 41) if case == "text" else datagen.random_bytes(600_000, 42)
    blocks, offs = _blocks_of(data, 2)
    bwt = b"".join(O.orc_bwt(blocks[offs[b]:offs[b + 1]])[0] for b in range(len(offs) - 1))
    got, freq = gpu_mtf(bwt, offs)
    for b in range(len(offs) - 1):
        mv, fr, nu = O.orc_mtf(bwt[offs[b]:offs[b + 1]])
        assert np.array_equal(got[b], mv), (case, b)
        assert np.array_equal(freq[b][: nu + 2].astype(np.int64), fr[: nu + 2].astype(np.int64)), (case, b)


def test_mtf_mixed_entropy_chunks():
    """Chunks on both MTF paths in one block (k_mtf_run: few distinct symbols; k_mtf_row: many)
    with zero runs crossing slice and chunk boundaries on the row path: text and random
    segments of a few kB, random bytes repeated 1..5 times, a 70-symbol alphabet."""
    rng = np.random.default_rng(77)
    parts = []
    for i in range(60):
        k = int(rng.integers(500, 6000))
        if i % 3 == 0:
            parts.append(datagen.text(k, 1000 + i))
        elif i % 3 == 1:
            v = rng.integers(0, 256, k // 3, dtype=np.uint8)
            parts.append(np.repeat(v, rng.integers(1, 6, v.size)).tobytes())
        else:
            parts.append(rng.integers(0, 70, k, dtype=np.uint8).tobytes())
    data = b"".join(parts)
    blocks, offs = _blocks_of(data, 1)
    bwt = b"".join(O.orc_bwt(blocks[offs[b]:offs[b + 1]])[0] for b in range(len(offs) - 1))
    got, freq = gpu_mtf(bwt, offs)
    for b in range(len(offs) - 1):
        mv, fr, nu = O.orc_mtf(bwt[offs[b]:offs[b + 1]])
        assert np.array_equal(got[b], mv), b
        assert np.array_equal(freq[b][: nu + 2].astype(np.int64), fr[: nu + 2].astype(np.int64)), b
    # raw random-ish columns straight into the MTF stage (not a BWT: every chunk high-entropy)
    raw = rng.integers(0, 256, 300_000, dtype=np.uint8)
    raw[1000:5000] = 7  # one long zero run across slices and chunks
    raw = raw.tobytes()
    offs2 = [0, 100_000, 100_001, 300_000]
    got, _ = gpu_mtf(raw, offs2)
    for b in range(3):
        mv, _, _ = O.orc_mtf(raw[offs2[b]:offs2[b + 1]])
        assert np.array_equal(got[b], mv), b


def test_mtf_long_zero_runs():
    # runs of identical BWT symbols spanning many MTF chunks (RUNA/RUNB carry across chunks)
    bwt = b"a" * 5000 + b"b" + b"a" * 3000 + b"c" * 70000 + b"ab" * 10
    offs = [0, len(bwt)]
    got, _ = gpu_mtf(bwt, offs)
    mv, _, _ = O.orc_mtf(bwt)
    assert np.array_equal(got[0], mv)


# ------------------------------------------------------------------ whole streams
@pytest.mark.parametrize("i,level", [(1, 1), (2, 2), (3, 3)])
def test_golden_samples(i, level):
    assert B.buff_to_buff_compress(gold(f"sample{i}.ref"), level) == gold(f"sample{i}.bz2")


@pytest.mark.parametrize("level", list(range(1, 10)))
def test_levels_vs_reference(level):
    data = datagen.text(1_200_000, 50 + level) + datagen.random_bytes(300_000, level)
    assert B.buff_to_buff_compress(data, level) == expected(data, level)


@pytest.mark.parametrize("data", [b"", b"a", b"aa", b"ab", b"abc" * 7 + b"d", bytes(range(256)) * 4,
                                  b"hello world " * 5000])
def test_edge_streams(data):
    for level in (1, 9):
        assert B.buff_to_buff_compress(data, level) == expected(data, level)


@pytest.mark.parametrize("c", [0x00, 0x61, 0xFB, 0xFF])
def test_single_byte_periodic_blocks(c):
    """Config 4 shape at -1: full blocks are (c c c c 0xFB)^k, exactly periodic (A5)."""
    data = bytes([c]) * 6_000_000
    assert B.buff_to_buff_compress(data, 1) == expected(data, 1)


def test_periodic_text_blocks():
    w = datagen.text(3_001, 99)
    for data in (w * 300, b"abcabcabd" * 120_000, b"ab" * 500_000):
        assert B.buff_to_buff_compress(data, 2) == expected(data, 2)


def _quasi_periodic_blocks(seed):
    """Blocks w^k w' (w' a proper prefix of w): the analytic path of qsa.h, beside ordinary
    blocks in the same batch."""
    rng = random.Random(seed)
    parts = [bytes([0x61] * 4 + [0xFB]) * 20_000 + b"a", bytes([0] * 4 + [0xFB]) * 7 + b"\0\0\0",
             datagen.text(30_000, 3)]
    for _ in range(24):
        w = bytes(rng.randrange(rng.choice([2, 3, 4, 256])) for _ in range(rng.randint(2, 256)))
        k = rng.randint(2, max(2, 150_000 // len(w)))
        parts.append(w * k + w[: rng.randint(1, len(w) - 1)])
    offs = [0]
    for p_ in parts:
        offs.append(offs[-1] + len(p_))
    return b"".join(parts), offs


def test_bwt_quasi_periodic_blocks():
    """Quasi-periodic blocks through the stage ABI (device detection k_qperiod, host plan,
    k_qsa) against the oracle, and the host analytic path (bzg_qperiodic_bwt) agrees."""
    blocks, offs = _quasi_periodic_blocks(9)
    bwt, orig = gpu_bwt(blocks, offs)
    nq = 0
    for b in range(len(offs) - 1):
        blk = blocks[offs[b]:offs[b + 1]]
        L, o, per = O.orc_bwt(blk)
        assert bwt[offs[b]:offs[b + 1]] == L, b
        assert orig[b] == o, b
        q = B.qperiodic_bwt(blk)
        if q is not None:
            nq += 1
            assert q[1:] == (L, o), b
    assert nq >= 20


@pytest.mark.parametrize("level", [1, 9])
def test_single_byte_quasi_periodic_tail(level):
    """Config 4 shape: a repeated byte whose last RLE1 chunk holds 1..3 bytes makes the last
    block (c c c c 0xFB)^k c.. quasi-periodic (k_qsa); full blocks stay exactly periodic (A5)."""
    for c, r in ((0x61, 1), (0xFB, 3), (0x00, 2)):
        data = bytes([c]) * (255 * 9_000 + r)
        assert B.buff_to_buff_compress(data, level) == expected(data, level), (c, r)


def test_single_byte_aperiodic_tail():
    # one symbol per block: period-1 blocks take origPtr 0 (blocksort.c:1349)
    for c in (0x00, 0xFB):
        data = bytes([c]) * 700
        assert B.buff_to_buff_compress(data, 1) == expected(data, 1)


def test_streaming_run_finish_edge():
    edge = bytes((i * 7 + (i >> 8)) % 251 + 1 for i in range(99_982))
    if not O.has_ref():
        pytest.skip("needs oracle/_ref for the streaming reference")
    for fin in (False, True):
        got = B.stream_compress([edge], 1, finish_with_last=fin)
        assert got == O.ref_stream_compress([edge], 1, finish_with_last=fin), fin


def test_streaming_chunked_and_flush():
    if not O.has_ref():
        pytest.skip("needs oracle/_ref for the streaming reference")
    data = datagen.text(700_000, 61)
    chunks = [data[i:i + 5000] for i in range(0, len(data), 5000)]
    assert B.stream_compress(chunks, 1) == O.ref_stream_compress(chunks, 1)
    chunks = [data[:250_000], data[250_000:400_000], data[400_000:]]
    assert B.stream_compress(chunks, 2, flush_after=(0, 1)) == O.ref_stream_compress(chunks, 2, flush_after=(0, 1))


def test_streaming_emits_blocks_as_they_fill():
    """BZ_RUN output appears about when the reference would emit it (bzlib.c:383-386): the
    first complete blocks come back after about two blocks of input, not after the whole
    staging limit; the whole stream still equals the reference's."""
    if not O.has_ref():
        pytest.skip("needs oracle/_ref for the streaming reference")
    data = datagen.text(6_000_000, 62)
    chunks = [data[i:i + 5000] for i in range(0, len(data), 5000)]
    prog = []
    got = B.stream_compress(chunks, 1, progress=prog)
    assert got == O.ref_stream_compress(chunks, 1)
    first = next(inp for inp, outb in prog if outb > 0)
    assert first <= 400_000, first  # -1 blocks hold ~100 kB: output after ~2-4 blocks of input
    half = next(outb for inp, outb in prog if inp >= len(data) // 2)
    assert half >= len(got) // 4, (half, len(got))  # output keeps pace in the middle


def test_concurrent_streams_four_threads():
    """Four host threads at once, each running BZ2_bzBuffToBuffCompress and chunked
    BZ2_bzCompress loops on its own inputs (the reference is reentrant per bz_stream,
    bzlib.c:144-207): every output equals the reference's for that thread's input."""
    import threading

    if not O.has_ref():
        pytest.skip("needs oracle/_ref for the streaming reference")
    inputs = [datagen.text(1_300_000 + 97_000 * t, 300 + t) + datagen.random_bytes(50_000 * t, t) for t in range(4)]
    want_b2b = [O.ref_compress(x, 1 + t) for t, x in enumerate(inputs)]
    chunks = [[x[i:i + 70_000] for i in range(0, len(x), 70_000)] for x in inputs]
    want_stream = [O.ref_stream_compress(c, 9 - t) for t, c in enumerate(chunks)]
    errors = []

    def work(t):
        try:
            for _ in range(3):
                got = B.buff_to_buff_compress(inputs[t], 1 + t)
                assert got == want_b2b[t], f"thread {t}: BuffToBuff differs"
                got = B.stream_compress(chunks[t], 9 - t)
                assert got == want_stream[t], f"thread {t}: bzCompress differs"
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(repr(e))

    ths = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors


def test_device_oom_is_mem_error():
    """A device allocation failure is BZ_MEM_ERROR (not BZ_OUTBUFF_FULL, which would tell a
    BuffToBuff caller to retry with a bigger destination); a short destination is
    BZ_OUTBUFF_FULL."""
    data = datagen.text(300_000, 5)
    L = B.lib()
    dst = ctypes.create_string_buffer(100)
    dl = ctypes.c_uint(100)
    assert L.BZ2_bzBuffToBuffCompress(dst, ctypes.byref(dl), data, len(data), 9, 0, 30) == B.BZ_OUTBUFF_FULL
    torch = pytest.importorskip("torch")
    n = 1_200_000_000
    d_in = torch.zeros(n, dtype=torch.uint8, device="cuda")  # real buffers: kernels that run read in bounds
    cap = B.bound(n)
    d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    B.lib().bzg_release()
    hog = []
    try:
        for chunk in (8 << 30, 1 << 30, 128 << 20):  # leave the engine no room for its workspace
            while True:
                try:
                    hog.append(torch.empty(chunk, dtype=torch.uint8, device="cuda"))
                except RuntimeError:
                    break
        st = B.bzg_stream_state()
        L.bzg_stream_init(ctypes.byref(st), 9)
        ob, cons = ctypes.c_uint64(0), ctypes.c_uint64(0)
        rc = L.bzg_compress_device(ctypes.c_void_p(d_in.data_ptr()), n, B.BZG_FLAG_END_SEGMENT | B.BZG_FLAG_TRAILER,
                                   ctypes.byref(st), ctypes.c_void_p(d_out.data_ptr()), cap, ctypes.byref(ob),
                                   ctypes.byref(cons), None)
        assert rc == B.BZ_MEM_ERROR, rc
    finally:
        del hog
        torch.cuda.empty_cache()
    del d_in, d_out
    torch.cuda.empty_cache()
    assert B.buff_to_buff_compress(data, 9) == expected(data, 9)  # the engine recovers


def test_file_api_write_matches_reference(tmp_path):
    """BZ2_bzWriteOpen / BZ2_bzWrite in 5000-byte pieces (the CLI's pattern, bzip2.c:329-427) /
    BZ2_bzWriteClose64 write the reference's RUN...FINISH stream; BZ2_bzopen("w") / bzwrite /
    bzclose likewise at -9."""
    if not O.has_ref():
        pytest.skip("needs oracle/_ref for the streaming reference")
    from tests.test_abi import _file_api, _libc

    L = _file_api(B.lib())
    L.BZ2_bzWrite.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    u = ctypes.POINTER(ctypes.c_uint)
    L.BZ2_bzWriteClose64.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_void_p, ctypes.c_int, u, u, u, u]
    L.BZ2_bzwrite.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    data = datagen.text(1_234_567, 77)
    pieces = [data[i:i + 5000] for i in range(0, len(data), 5000)]
    c = _libc()
    p = tmp_path / "w.bz2"
    f = c.fopen(str(p).encode(), b"wb")
    e = ctypes.c_int(0)
    h = L.BZ2_bzWriteOpen(ctypes.byref(e), f, 3, 0, 0)
    assert h and e.value == B.BZ_OK
    for x in pieces:
        L.BZ2_bzWrite(ctypes.byref(e), h, x, len(x))
        assert e.value == B.BZ_OK
    cnt = [ctypes.c_uint(0) for _ in range(4)]
    L.BZ2_bzWriteClose64(ctypes.byref(e), h, 0, *[ctypes.byref(x) for x in cnt])
    assert e.value == B.BZ_OK
    c.fclose(f)
    want = O.ref_stream_compress(pieces, 3)
    assert p.read_bytes() == want
    assert (cnt[0].value, cnt[1].value, cnt[2].value, cnt[3].value) == (len(data), 0, len(want), 0)
    q = tmp_path / "z.bz2"
    b = L.BZ2_bzopen(str(q).encode(), b"w9")
    for x in pieces:
        assert L.BZ2_bzwrite(b, x, len(x)) == len(x)
    L.BZ2_bzclose(b)
    assert q.read_bytes() == O.ref_stream_compress(pieces, 9)


@pytest.mark.parametrize("level", [1, 9])
def test_multi_device_host_path(monkeypatch, level):
    """BZ2_bzBuffToBuffCompress over several engines in one process (BZG_DEVICES=0,0,0: three
    engines on this box's GPU; the 8-GPU node uses BZG_NGPUS=8): chunk maps per shard, the cut
    chain, owned block ranges, bit-shifted copies behind each other, combined CRC and trailer
    give the reference's stream."""
    rnd = random.Random(level)
    txt = datagen.text(14_000_000, 0x5EED0011)
    cases = {
        "text": txt,
        "text_run_text": txt[:5_000_000] + b"q" * 9_000_000 + txt[5_000_000:9_000_000],
        "one_byte": b"z" * 30_000_000,  # one run over every shard boundary
        "runs_of_4": b"aaaabbbb" * 1_600_000,
        "random": datagen.random_bytes(13_000_000, 5),
        "mixed_runs": bytes(np.repeat(np.frombuffer(datagen.random_bytes(200_000, 9), np.uint8) % 3,
                                      np.random.default_rng(3).integers(1, 300, 200_000)).tobytes()[:13_000_000]),
    }
    monkeypatch.setenv("BZG_DEVICES", "0,0,0")
    for name, data in cases.items():
        got = B.buff_to_buff_compress(data, level)
        assert got == expected(data, level), name
    monkeypatch.setenv("BZG_DEVICES", "0,0,0,0")  # a stream whose last byte opens no block
    data = b"a" * (255 * 19996 * 3 + 4) + b"b"
    assert B.buff_to_buff_compress(data, 1) == expected(data, 1)
    monkeypatch.setenv("BZG_DEVICES", "0,0,0,0,0,0")  # more repeats than engines per device: clamped
    assert B.buff_to_buff_compress(txt, level) == expected(txt, level)


@pytest.mark.parametrize("plan", [None, "100,100", "64,64,64"])
def test_host_pipelined_equals_device(monkeypatch, plan):
    """BZ2_bzBuffToBuffCompress of a large host buffer runs as a pipeline (engine.hip
    host_call_pipelined: piece uploads, the pieces' front and back stages over two workspace
    slots, downloads overlapped); its bytes equal one device-resident call on the same input,
    for the default piece plan and for 3 and 4 pieces (BZG_H2H_PLAN), and a short destination
    gives BZ_OUTBUFF_FULL."""
    torch = pytest.importorskip("torch")
    if plan:
        monkeypatch.setenv("BZG_H2H_PLAN", plan)
    data = datagen.text(300_000_000, 404) + datagen.random_bytes(20_000_000, 5) + b"z" * 30_000_000
    got = B.buff_to_buff_compress(data, 9)
    d_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
    cap = B.bound(len(data))
    d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    nb, cons, _ = B.compress_device(d_in.data_ptr(), len(data), 9, d_out.data_ptr(), cap,
                                    stream_ptr=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert cons == len(data) and got == d_out[:nb].cpu().numpy().tobytes()
    small = ctypes.create_string_buffer(len(got) // 2)
    dl = ctypes.c_uint(len(got) // 2)
    assert B.lib().BZ2_bzBuffToBuffCompress(small, ctypes.byref(dl), data, len(data), 9, 0, 30) == B.BZ_OUTBUFF_FULL


def test_round_trip_large_properties():
    """At bench-like sizes: decode(encode(x)) == x with the system bzip2 decoder, and the
    stream equals the reference's on a 4 MB slice."""
    data = datagen.text(24_000_000, 71)
    comp = B.buff_to_buff_compress(data, 9)
    assert bz2.decompress(comp) == data
    sl = data[:4_000_000]
    assert B.buff_to_buff_compress(sl, 9) == expected(sl, 9)


def _chunks(buf, size):
    mv = memoryview(buf)
    return (mv[i:i + size] for i in range(0, len(buf), size))


def test_full_size_single_byte_4gib():
    """BASELINE config 4 at full size: 4 GiB of one byte through chunked BZ2_bzCompress (u32
    limits, long-run RLE1, periodic blocks): the whole stream equals, byte for byte, the
    reference's own BZ2_bzCompress driven with the same 256 MiB RUN chunks and FINISH (about 11 s
    of one core), and the system decoder returns the input exactly."""
    n = 1 << 32
    data = b"a" * n
    comp = B.stream_compress(_chunks(data, 1 << 28), 9, out_chunk=1 << 24)
    assert comp == O.ref_stream_compress(_chunks(data, 1 << 28), 9)
    out = bz2.decompress(comp)
    assert len(out) == n and out == data


def test_full_size_random_4gib_properties():
    """BASELINE config 5 at full size: 4 GiB of PRNG bytes.  Its first 512 MiB byte for byte
    against the reference's BZ2_bzCompress under the same chunking (about 25 s of one core); for
    the whole 4 GiB (the reference run would take minutes) properties: output size of an incompressible stream
    (about 1.0044 x input); the whole stream decodes back to the input on the GPU decoder
    (every block CRC and the combined CRC checked), and its first 256 MiB also through the
    system decoder (an independent implementation)."""
    torch = pytest.importorskip("torch")
    n = 1 << 32
    data = np.random.default_rng(0x5EED0005).integers(0, 256, size=n, dtype=np.uint8).tobytes()
    # byte-exact on a 512 MiB prefix: the same chunked call pattern through the reference
    pre = memoryview(data)[: 1 << 29]
    assert B.stream_compress(_chunks(pre, 1 << 28), 9, out_chunk=1 << 24) == O.ref_stream_compress(_chunks(pre, 1 << 28), 9)
    del pre
    comp = B.stream_compress(_chunks(data, 1 << 28), 9, out_chunk=1 << 24)
    assert 1.003 < len(comp) / n < 1.006
    d = bz2.BZ2Decompressor()
    head = d.decompress(comp, max_length=1 << 28)
    assert head == data[: 1 << 28]
    del head, d
    d_comp = torch.frombuffer(bytearray(comp), dtype=torch.uint8).to("cuda")
    del comp
    d_out = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    rc, got = B.decompress_device(d_comp.data_ptr(), d_comp.numel(), d_out.data_ptr(), n + 64,
                                  stream_ptr=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert rc == B.BZ_OK and got == n
    d_ref = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
    assert torch.equal(d_out[:n], d_ref)


def test_device_api_with_torch_buffers():
    torch = pytest.importorskip("torch")
    data = datagen.text(3_000_000, 81)
    d_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
    cap = B.bound(len(data))
    d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    nbytes, consumed, _ = B.compress_device(d_in.data_ptr(), len(data), 9, d_out.data_ptr(), cap,
                                            stream_ptr=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert consumed == len(data)
    assert bytes(d_out[:nbytes].cpu().numpy().tobytes()) == expected(data, 9)


def test_device_api_split_batches_unaligned_output():
    """One bzg_compress_device call larger than the engine's batch limit (1.5e9 bytes): the
    input is cut into batches inside the call and each batch's bits land right behind the
    previous batch's bytes, whatever their alignment; also a caller output pointer that is not
    4-byte aligned."""
    torch = pytest.importorskip("torch")
    data = datagen.text(2_000_000, 93)
    d_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
    cap = B.bound(len(data))
    buf = torch.zeros(cap + 8, dtype=torch.uint8, device="cuda")
    nb, cons, _ = B.compress_device(d_in.data_ptr(), len(data), 9, buf.data_ptr() + 3, cap)
    torch.cuda.synchronize()
    assert cons == len(data) and buf[3:3 + nb].cpu().numpy().tobytes() == expected(data, 9)
    n = 1_600_000_000  # two batches; RLE1 makes it 1.6e9 * 5 / 255 block bytes
    d_in = torch.full((n,), 0x61, dtype=torch.uint8, device="cuda")
    cap = B.bound(n)
    out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    nb, cons, _ = B.compress_device(d_in.data_ptr(), n, 9, out.data_ptr(), cap)
    torch.cuda.synchronize()
    assert cons == n
    got = out[:nb].cpu().numpy().tobytes()
    del d_in, out
    torch.cuda.empty_cache()
    assert got == expected(b"a" * n, 9)


_PIPE_CHILD = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
import bzip2_amd as B
data = open(sys.argv[2], "rb").read()
d_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
cap = B.bound(len(data))
out = torch.zeros(cap + 8, dtype=torch.uint8, device="cuda")
nb, cons, _ = B.compress_device(d_in.data_ptr(), len(data), 9, out.data_ptr() + int(sys.argv[4]), cap)
torch.cuda.synchronize()
assert cons == len(data), cons
open(sys.argv[3], "wb").write(out[int(sys.argv[4]):int(sys.argv[4]) + nb].cpu().numpy().tobytes())
s = B.last_stats()
print(s["nblocks"], flush=True)
"""


@pytest.mark.parametrize("offset", [0, 1])
def test_device_api_pipelined_batches(tmp_path, offset):
    """A multi-batch device call runs its batches as a pipeline (Engine::compress_pipelined: the
    MTF / tables / packing of batch j beside the RLE1 and sorts of batch j + 1, two workspace
    slots).  With the batch limit lowered to 12 MB (BZG_MAX_BATCH, in a child process: the limit
    is read once per process), 40 MB of text is 4 batches; the stream must equal the
    reference's and the sequential batches' (BZG_BATCH_PIPE=0), at an aligned and an odd output
    pointer."""
    import subprocess
    import sys

    data = datagen.text(40_000_000, 97)
    src = tmp_path / "in.bin"
    src.write_bytes(data)
    outs = {}
    for pipe in ("1", "0"):
        dst = tmp_path / f"out{pipe}.bin"
        env = dict(os.environ, BZG_MAX_BATCH="12000000", BZG_BATCH_PIPE=pipe)
        r = subprocess.run([sys.executable, "-c", _PIPE_CHILD, ROOT, str(src), str(dst), str(offset)], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs[pipe] = dst.read_bytes()
    assert outs["1"] == outs["0"]
    assert outs["1"] == expected(data, 9)


def test_device_api_continuation_batches():
    """Non-final batches (RUN semantics) + a final batch give the RUN-then-FINISH stream."""
    torch = pytest.importorskip("torch")
    data = datagen.text(2_600_000, 91)
    d_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
    cap = B.bound(len(data))
    d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    st = B.bzg_stream_state()
    B.lib().bzg_stream_init(ctypes.byref(st), 1)
    out = bytearray()
    pos = 0
    for piece in (700_000, 900_000):
        nb, cons, st = B.compress_device(d_in.data_ptr() + pos, piece, 1, d_out.data_ptr(), cap, flags=0, state=st)
        out += d_out[:nb].cpu().numpy().tobytes()
        pos += cons
    nb, cons, st = B.compress_device(d_in.data_ptr() + pos, len(data) - pos, 1, d_out.data_ptr(), cap,
                                     flags=B.BZG_FLAG_END_SEGMENT | B.BZG_FLAG_TRAILER, state=st)
    out += d_out[:nb].cpu().numpy().tobytes()
    assert bytes(out) == O.orc_compress(data, 1, tail_merge=0)


# ------------------------------------------------------------------ one stream sharded
def _shard_inputs():
    from tests.test_shard import _inputs

    d = _inputs()
    d["text_big"] = datagen.text(6_000_000, 93)
    return d


@pytest.mark.parametrize("level", [1, 9])
def test_seg_walk_chain_matches_whole_stream_cuts(level):
    """bzg_seg_map / bzg_seg_walk (device) through the rank chain of bzip2_amd.shard, run locally
    shard after shard, against the whole-stream cut rule (tests/shard_cpu.py, pinned to the
    oracle's blocks in test_shard.py)."""
    torch = pytest.importorskip("torch")
    from bzip2_amd import shard as S
    from tests.shard_cpu import cuts_whole

    rnd = random.Random(level)
    for name, data in _shard_inputs().items():
        want = cuts_whole(data, level)
        n = len(data)
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
        be = S.GpuBackend(level)
        for trial in range(3):
            k = rnd.choice([1, 2, 4, 8])
            bnd = [0] + sorted(rnd.sample(range(1, n), k - 1)) + [n]
            msg, cuts = None, []
            for r, (a, b) in enumerate(zip(bnd, bnd[1:])):
                c, msg = S.chain_piece(be, t[a:b], a, n, msg, final=(r == len(bnd) - 2))
                cuts += c
            assert cuts == want, (name, level, bnd)


def _gpu_shard_worker(rank, world, port, cases, out):
    import torch
    import torch.distributed as dist

    from bzip2_amd import shard as S

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        for key, (data, level, bnd) in cases.items():
            t = torch.frombuffer(bytearray(data[bnd[rank]:bnd[rank + 1]]), dtype=torch.uint8).to("cuda")
            res = S.compress_sharded(t, bnd[rank], len(data), level)
            torch.cuda.synchronize()
            if rank == 0:
                out[key] = res.cpu().numpy().tobytes()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 3])
def test_sharded_stream_on_device(world):
    """compress_sharded with the GPU backend (HIP path for cuts and compression), ranks sharing
    cuda:0 over gloo: rank 0's stream equals the reference's stream of the whole input."""
    import socket

    import torch.multiprocessing as mp

    rnd = random.Random(100 + world)
    cases = {}
    for name, data in _shard_inputs().items():
        n = len(data)
        for level in (1, 9):
            bnd = [0] + sorted(rnd.sample(range(1, n), world - 1)) + [n]
            cases[(name, level)] = (data, level, bnd)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = mp.get_context("spawn").Manager().dict()
    mp.spawn(_gpu_shard_worker, args=(world, port, cases, out), nprocs=world, join=True)
    for key, (data, level, bnd) in cases.items():
        assert out[key] == expected(data, level), (key, bnd)


def _gpu_shard_big_worker(rank, world, port, out):
    import torch
    import torch.distributed as dist

    from bzip2_amd import shard as S

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cases = {
            # one run across every shard boundary (the host run arithmetic over 255-byte chunks)
            "byte_a": (lambda: torch.full((200_000_000,), 0x61, dtype=torch.uint8, device="cuda"), 9),
            "text": (lambda: torch.frombuffer(bytearray(datagen.text(60_000_000, 0x5EED0003)),
                                              dtype=torch.uint8).to("cuda"), 9),
        }
        for key, (make, level) in cases.items():
            full = make()
            n = full.numel()
            bnd = [n * r // world for r in range(world + 1)]
            if key == "text":  # a boundary right inside the first block's last run of bytes
                bnd[1] = 899_000
            res = S.compress_sharded(full[bnd[rank]:bnd[rank + 1]], bnd[rank], n, level)
            torch.cuda.synchronize()
            if rank == 0:
                out[key] = res.cpu().numpy().tobytes()
            del full
    finally:
        dist.destroy_process_group()


def test_sharded_stream_on_device_large():
    """Three ranks on one GPU over gloo: 200 MB of one byte and 60 MB of text at -9, sharded,
    against the reference's stream of the whole input."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = mp.get_context("spawn").Manager().dict()
    mp.spawn(_gpu_shard_big_worker, args=(3, port, out), nprocs=3, join=True)
    assert out["byte_a"] == expected(b"a" * 200_000_000, 9)
    assert out["text"] == expected(datagen.text(60_000_000, 0x5EED0003), 9)


def _gpu_shard_1g_worker(rank, world, port, out):
    import torch
    import torch.distributed as dist

    from bzip2_amd import shard as S

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 1_000_000_000
        data = datagen.text(n, 0x5EED0003)  # every rank generates the stream (seconds, in parallel)
        bnd = [n * r // world for r in range(world + 1)]
        t = torch.frombuffer(bytearray(data[bnd[rank]:bnd[rank + 1]]), dtype=torch.uint8).to("cuda")
        res = S.compress_sharded(t, bnd[rank], n, 9)
        torch.cuda.synchronize()
        if rank == 0:
            got = res.cpu().numpy().tobytes()
            want = expected(data, 9)  # the reference build, about 35 s of one core
            out["len"] = len(got)
            out["eq"] = got == want
    finally:
        dist.destroy_process_group()


def test_sharded_stream_1gb_config3():
    """BASELINE config 3's path at its full size: 1e9 bytes of enwik9-class text at -9 sharded
    over three ranks (gloo, all on this box's one GPU) through compress_sharded; rank 0's
    gathered stream equals the reference's BZ2_bzBuffToBuffCompress of the whole 1e9 bytes."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = mp.get_context("spawn").Manager().dict()
    mp.spawn(_gpu_shard_1g_worker, args=(3, port, out), nprocs=3, join=True)
    assert out["eq"], out["len"]


def _nccl_worker(rank, world, port, out):
    import torch
    import torch.distributed as dist

    from bzip2_amd import shard as S

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    try:
        data = datagen.text(30_000_000, 0x5EED0004) + b"x" * 5_000_000
        n = len(data)
        bnd = [n * r // world for r in range(world + 1)]
        t = torch.frombuffer(bytearray(data[bnd[rank]:bnd[rank + 1]]), dtype=torch.uint8).to("cuda")
        res = S.compress_sharded(t, bnd[rank], n, 9)  # device tensors through RCCL send/recv
        torch.cuda.synchronize()
        if rank == 0:
            out["eq"] = res.cpu().numpy().tobytes() == expected(data, 9)
    finally:
        dist.destroy_process_group()


@pytest.mark.skipif(not __import__("torch").cuda.is_available() or __import__("torch").cuda.device_count() < 2,
                    reason="the RCCL path needs two GPUs (one rank per GPU)")
def test_sharded_stream_nccl_two_gpus():
    """compress_sharded's device-tensor branch (RCCL send/recv/all_gather into slices of the
    result), one rank per GPU."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = mp.get_context("spawn").Manager().dict()
    mp.spawn(_nccl_worker, args=(2, port, out), nprocs=2, join=True)
    assert out["eq"]


# ------------------------------------------------------------------ block boundaries
def test_find_magics_matches_scan():
    """bzg_find_magics against the CPU restatement of the bzip2recover scan (tests/magic_ref.py)
    on real streams (many blocks at -1), planted magics at every bit shift (stream start and
    end included), odd lengths and a misaligned device pointer."""
    torch = pytest.importorskip("torch")
    from tests import magic_ref as M

    rnd = random.Random(17)
    cases = [O.orc_compress(datagen.text(2_000_000, 23) + b"y" * 500_000, 1), b"", b"\x31\x41"]
    for n in (7, 64, 4099, 100_003):
        slots = rnd.sample(range(1, max(2, (8 * n - 48) // 64 - 1)), min(30, max(1, (8 * n - 48) // 64 - 2)))
        planted = [(64 * s + rnd.randrange(8), rnd.randrange(2)) for s in slots if 64 * s + 55 < 8 * n]
        if n >= 6:
            planted += [(0, 0), (8 * n - 48, 1)]
        cases.append(M.plant(n, sorted(set(planted)), n))
    for data in cases:
        want = M.scan(data)
        for shift in (0, 3):
            buf = torch.zeros(len(data) + 16, dtype=torch.uint8, device="cuda")
            if data:
                buf[shift:shift + len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
            got = B.find_magics(buf.data_ptr() + shift, len(data))
            assert got == want, (len(data), shift)


def test_find_magics_full_size_rate():
    """A 1 GB buffer with a magic every 900 kB: every one found; the scan's rate is printed
    (HBM-bound: 1 byte read per byte)."""
    torch = pytest.importorskip("torch")
    n = 1_000_000_000
    buf = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    offs = list(range(8 * 1000, 8 * n - 64, 8 * 900_007 + 3))
    pat = [(0x314159265359 >> (47 - i)) & 1 for i in range(48)]
    for o in offs:  # write each magic's bits on the host side of a small window
        lo, hi = o // 8, (o + 48 + 7) // 8 + 1
        w = np.unpackbits(buf[lo:hi].cpu().numpy())
        w[o - 8 * lo:o - 8 * lo + 48] = pat
        buf[lo:hi] = torch.from_numpy(np.packbits(w)).to("cuda")
    B.find_magics(buf.data_ptr(), n)  # warm-up
    torch.cuda.synchronize()
    import time

    t = time.perf_counter()
    got = B.find_magics(buf.data_ptr(), n)
    dt = time.perf_counter() - t
    assert set(offs) <= {o for o, k in got if k == 0}  # chance magics in random bytes: p ~ 1e-4
    print(f"\nbzg_find_magics: {n / dt / 1e9:.1f} GB/s over {n} B ({len(got)} magics)")
