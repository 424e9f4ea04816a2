"""Test infrastructure: CPU restatement of the bzip2recover.c:360-395 magic scan (every bit
offset where the 48-bit block-header magic 0x314159265359 or end-of-stream magic 0x177245385090
starts; bzip2recover.c:284-288), in numpy, as the checker for bzg_find_magics."""
import numpy as np

MAGIC_BLOCK = 0x314159265359
MAGIC_EOS = 0x177245385090


def scan(data: bytes):
    """Sorted [(bit_offset, kind)] with kind 0 = block header, 1 = end of stream."""
    n = len(data)
    if n == 0:
        return []
    padded = np.frombuffer(bytes(data) + b"\0" * 8, dtype=np.uint8)
    win = np.lib.stride_tricks.as_strided(padded[:8].view(">u8"), shape=(n,), strides=(1,)).astype(np.uint64)
    out = []
    for k in range(8):
        v = (win >> np.uint64(16 - k)) & np.uint64((1 << 48) - 1)
        for magic, kind in ((MAGIC_BLOCK, 0), (MAGIC_EOS, 1)):
            pos = np.flatnonzero(v == np.uint64(magic)).astype(np.int64) * 8 + k
            out += [(int(p), kind) for p in pos if p + 48 <= 8 * n]
    return sorted(out)


def plant(n: int, offsets_kinds, seed: int) -> bytes:
    """Random bytes with the given magics written at the given bit offsets."""
    rng = np.random.default_rng(seed)
    bits = np.unpackbits(rng.integers(0, 256, n, dtype=np.uint8))
    for off, kind in offsets_kinds:
        m = MAGIC_EOS if kind else MAGIC_BLOCK
        bits[off:off + 48] = [(m >> (47 - i)) & 1 for i in range(48)]
    return np.packbits(bits).tobytes()
