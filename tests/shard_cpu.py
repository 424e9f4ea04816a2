"""Test infrastructure: a CPU stand-in for the GPU backend of bzip2_amd.shard (checker only).

`chunks`/`cuts_whole` restate the block-cut rule of bzlib.c:211-315 (RLE1 chunks of <= 255 equal
bytes; a block ends once it holds >= nblockMAX RLE1 bytes; in FINISH the last input byte never
starts a block, bzlib.c:276-308, 361-396) in numpy; they are pinned against the oracle's block
sizes (oracle/bz_oracle.c orc_rle1) in tests/test_shard.py.  `CpuBackend.compress` takes the
oracle's whole-stream output of a range and strips header / trailer to get the raw block bits.
"""
import numpy as np
import torch

from bzip2_amd.shard import TRAILER_MAGIC, nblock_max
from tests import oracles as O


def chunks(d: np.ndarray):
    """Input starts, lengths and RLE1 sizes of the chunks of d (starting at a chunk start)."""
    n = len(d)
    change = np.flatnonzero(d[1:] != d[:-1]) + 1
    rs = np.concatenate([[0], change]).astype(np.int64)
    re = np.concatenate([change, [n]]).astype(np.int64)
    k = (re - rs + 254) // 255
    first = np.cumsum(k) - k
    idx = np.arange(int(k.sum()), dtype=np.int64)
    starts = np.repeat(rs, k) + 255 * (idx - np.repeat(first, k))
    lens = np.minimum(255, np.repeat(re, k) - starts)
    return starts, lens, np.where(lens < 4, lens, 5)


def walk(starts, lens, sizes, level, fill, final):
    mx = nblock_max(level)
    assert fill < mx, "bzg_seg_walk rejects fill_in >= nblockMAX (BZ_PARAM_ERROR)"
    outpos = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    s = -fill
    cuts = []
    while True:
        i = int(np.searchsorted(outpos, s + mx, "left"))
        if i >= len(starts):
            break
        if final and i == len(starts) - 1 and lens[i] == 1:
            break
        cuts.append(int(starts[i]))
        s = int(outpos[i])
    return cuts, int(starts[-1]), int(outpos[-1] - s)


def cuts_whole(data: bytes, level: int):
    """Block start offsets (after 0) of the whole stream compressed with FINISH."""
    st, ln, sz = chunks(np.frombuffer(data, np.uint8))
    return walk(st, ln, sz, level, 0, True)[0]


def strip(stream: bytes, header: bool):
    """Raw block bits of an oracle stream: (uint8 tensor, nbits, combined CRC)."""
    bits = np.unpackbits(np.frombuffer(stream, np.uint8))
    n = len(bits)
    for pad in range(8):
        st = n - pad - 80
        if int("".join(map(str, bits[st:st + 48])), 2) == TRAILER_MAGIC and not bits[n - pad:].any():
            break
    else:
        raise AssertionError("no trailer")
    crc = int("".join(map(str, bits[st + 48:st + 80])), 2)
    payload = bits[(0 if header else 32):st]
    return torch.from_numpy(np.packbits(payload).copy()), len(payload), crc


class CpuBackend:
    def __init__(self, level: int):
        self.level = level
        self.calls = {"map": 0, "walk": 0, "compress": 0}

    def map_region(self, d: torch.Tensor) -> None:
        self.calls["map"] += 1
        self.c = chunks(d.cpu().numpy())

    def walk(self, fill: int, final: bool, n: int):
        self.calls["walk"] += 1
        return walk(*self.c, self.level, fill, final)

    def compress(self, d: torch.Tensor, header: bool, final: bool):
        self.calls["compress"] += 1
        data = d.cpu().numpy().tobytes()
        stream = O.orc_compress(data, self.level, 1 if final else 0)
        nblk = len(O.orc_rle1(data, self.level, 1 if final else 0)[1]) - 1
        bits, nbits, crc = strip(stream, header)
        return bits, nbits, nblk, crc
