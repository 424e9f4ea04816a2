"""The magic-scan checker (tests/magic_ref.py) on streams whose block layout the oracle knows,
and on planted magics.  The GPU scan (bzg_find_magics) is compared with it in test_gpu.py."""
import random

from tests import datagen, magic_ref as M, oracles as O


def test_scan_finds_every_block_of_oracle_streams():
    for level in (1, 3):
        data = datagen.text(700_000, 21) + b"x" * 300_000
        stream = O.orc_compress(data, level)
        found = M.scan(stream)
        nblocks = len(O.orc_rle1(data, level)[1]) - 1
        heads = [o for o, k in found if k == 0]
        eos = [o for o, k in found if k == 1]
        assert heads[0] == 32 and len(heads) >= nblocks
        assert eos and eos[-1] >= heads[-1]
        # the trailer: magic, 32-bit CRC, < 8 bits of padding
        assert 8 * len(stream) - 7 <= eos[-1] + 80 <= 8 * len(stream)


def test_scan_planted():
    rnd = random.Random(5)
    n = 4099
    slots = rnd.sample(range(1, (8 * n - 48) // 64 - 1), 40)  # one magic per 64-bit slot
    planted = sorted([(64 * s + rnd.randrange(8), rnd.randrange(2)) for s in slots] + [(0, 0), (8 * n - 48, 1)])
    data = M.plant(n, planted, 9)
    assert M.scan(data) == planted
