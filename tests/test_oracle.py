"""CPU tests: the oracle restatement (oracle/bz_oracle.c) pinned against the reference's own
golden vectors (sample{1,2,3}, reference Makefile:56-70) and -- where oracle/_ref was built --
against the reference library itself, stage by stage."""
import os
import random

import numpy as np
import pytest

from tests import datagen, oracles as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def gold(name):
    with open(os.path.join(GOLD, name), "rb") as f:
        return f.read()


@pytest.mark.parametrize("i,level", [(1, 1), (2, 2), (3, 3)])
def test_oracle_reproduces_reference_golden_samples(i, level):
    assert O.orc_compress(gold(f"sample{i}.ref"), level) == gold(f"sample{i}.bz2")


def test_crc_table_matches_reference():
    if not O.has_ref():
        pytest.skip("oracle/_ref not built")
    for i in range(256):
        assert O.orc().orc_crc_table(i) == O.ref().ref_crc_table_entry(i)


def test_huffman_tie_order_kat():
    # equal frequencies are broken by subtree depth
    assert O.orc_code_lengths([10] * 6) == [3, 3, 2, 3, 2, 3]


def test_huffman_rescale_kat():
    freq = [int(2 ** (i // 2)) if i < 40 else 1 for i in range(258)]
    ln = O.orc_code_lengths(freq)
    assert max(ln) == 17
    if O.has_ref():
        assert ln == O.ref_code_lengths(freq)


@pytest.mark.skipif(not O.has_ref(), reason="oracle/_ref not built")
def test_huffman_random_vs_reference():
    rng = random.Random(7)
    for _ in range(300):
        alpha = rng.randint(3, 258)
        mode = rng.random()
        if mode < 0.3:
            freq = [rng.randint(0, 5) for _ in range(alpha)]
        elif mode < 0.6:
            freq = [int(rng.paretovariate(1.1) * 10) for _ in range(alpha)]
        else:
            freq = [rng.randint(0, 900_000 // alpha) for _ in range(alpha)]
        # a table never sees more than nMTF <= 900,001 symbols, so weights stay in int32
        assert O.orc_code_lengths(freq) == O.ref_code_lengths(freq)


@pytest.mark.skipif(not O.has_ref(), reason="oracle/_ref not built")
def test_bwt_random_blocks_vs_reference():
    rng = random.Random(11)
    for _ in range(400):
        n = rng.randint(1, 300)
        alpha = rng.choice([1, 2, 3, 4, 26, 256])
        blk = bytes(rng.randrange(alpha) for _ in range(n))
        if rng.random() < 0.25:  # exactly periodic blocks (A5 through the resolver)
            w = blk[: rng.randint(1, 7)] or b"a"
            blk = w * rng.randint(2, 40)
        assert O.orc_bwt(blk)[:2] == O.ref_blocksort(blk)


@pytest.mark.skipif(not O.has_ref(), reason="oracle/_ref not built")
@pytest.mark.parametrize("level", [1, 9])
def test_oracle_matches_reference_streams(level):
    rng = random.Random(level)
    cases = [b"", b"a", b"aa", b"ab", b"abab" * 100, bytes(1000), b"hello world " * 5000,
             datagen.random_bytes(250_000, 3), datagen.text(400_000, 5), b"a" * 1_000_000, b"\xfb" * 300_000,
             b"abcabcabd" * 30000, bytes(rng.randrange(4) for _ in range(200_000))]
    for c in cases:
        assert O.orc_compress(c, level) == O.ref_compress(c, level), len(c)


@pytest.mark.skipif(not O.has_ref(), reason="oracle/_ref not built")
def test_run_then_finish_segmentation_edge():
    """a 99,982-byte input with no equal neighbours splits differently when
    the last byte arrives with BZ_RUN (2 blocks) than with BZ_FINISH (1 block)."""
    data = bytes((i * 7 + (i >> 8)) % 251 + 1 for i in range(99_982))
    assert all(data[i] != data[i + 1] for i in range(len(data) - 1))
    run = O.ref_stream_compress([data], 1)
    fin = O.ref_stream_compress([data], 1, finish_with_last=True)
    assert run != fin
    assert O.orc_compress(data, 1, tail_merge=0) == run
    assert O.orc_compress(data, 1, tail_merge=1) == fin
    _, offs_run, _ = O.orc_rle1(data, 1, 0)
    _, offs_fin, _ = O.orc_rle1(data, 1, 1)
    assert len(offs_run) == 3 and len(offs_fin) == 2


def test_rle1_chunking_rules():
    blocks, offs, crcs = O.orc_rle1(b"a" * 10 + b"b" * 3 + b"c" * 600 + b"d", 9)
    assert blocks == b"aaaa\x06bbbcccc\xfbcccc\xfbcccc\x56d"
    assert len(crcs) == 1


def test_mtf_kat():
    mtfv, freq, nu = O.orc_mtf(b"bbbaaac")
    # list a,b,c: b at 1 -> 2; run of 2 zeros -> RUNB; a at 1 -> 2; 2 zeros -> RUNB; c at 2 -> 3; EOB 4
    assert list(mtfv) == [2, 1, 2, 1, 3, 4]
    assert nu == 3
