"""Builds tests/golden/randomised.{bz2,out}: a .bz2 stream whose block is randomised (rand bit
1, the pre-0.9.5 encoder option the reference still decodes, bzlib_private.h:167-179).

X = 60,000 seeded random bytes with no run of 4 equal bytes, so RLE1 is the identity.  The
decoder XORs the walk output y with the mask bit at every position t = A_{k+1} - 2 (A the
running sum of the format's random-number table, bzip2_amd/csrc/rnums.inc), so the stream
carries the reference's -1 coding of y = X ^ mask with the rand bit set and the block /
combined CRCs of X.  The script checks with the reference build (oracle/_ref) that the
stream decodes to X.  Run from the repo root: python tests/golden/make_randomised.py"""
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tests import oracles as O  # noqa: E402


def rnums():
    src = open(os.path.join(ROOT, "bzip2_amd", "csrc", "rnums.inc")).read()
    src = "\n".join(l for l in src.splitlines() if not l.lstrip().startswith("//"))
    return [int(x) for x in re.findall(r"\d+", src)]


def crc32_bz(data: bytes) -> int:
    tab = []
    for i in range(256):
        r = i << 24
        for _ in range(8):
            r = ((r << 1) ^ 0x04C11DB7) if r & 0x80000000 else (r << 1)
        tab.append(r & 0xFFFFFFFF)
    c = 0xFFFFFFFF
    for b in data:
        c = ((c << 8) & 0xFFFFFFFF) ^ tab[(c >> 24) ^ b]
    return c ^ 0xFFFFFFFF


def has_run4(a: np.ndarray) -> bool:
    e = a[1:] == a[:-1]
    return bool((e[:-2] & e[1:-1] & e[2:]).any())


def main():
    n = 60000
    mask = np.zeros(n, dtype=np.uint8)
    acc = 0
    r = rnums()
    assert len(r) == 512
    k = 0
    while True:
        acc += r[k % 512]
        if acc - 2 >= n:
            break
        mask[acc - 2] = 1
        k += 1
    seed = 1
    while True:
        x = np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)
        y = x ^ mask
        if not has_run4(x) and not has_run4(y):
            break
        seed += 1
    X, Y = x.tobytes(), y.tobytes()
    s = bytearray(O.ref_compress(Y, 1))
    assert s[4:10] == bytes.fromhex("314159265359")
    crc = crc32_bz(X)
    s[10:14] = crc.to_bytes(4, "big")
    s[14] |= 0x80  # the rand bit follows the CRC
    # end-of-stream magic and combined CRC (= the one block's CRC) near the end
    bits = int.from_bytes(s, "big")
    nb = 8 * len(s)
    for pos in range(nb - 80, nb - 80 - 16, -1):
        if (bits >> (nb - pos - 48)) & ((1 << 48) - 1) == 0x177245385090:
            break
    else:
        raise SystemExit("no end-of-stream magic")
    sh = nb - (pos + 48) - 32
    bits &= ~(((1 << 32) - 1) << sh)
    bits |= crc << sh
    s = bytearray(bits.to_bytes(len(s), "big"))
    rc, out = O.ref_decompress(bytes(s), n + 100)
    assert rc == 0 and out == X, ("reference does not decode the fixture", rc)
    d = os.path.dirname(os.path.abspath(__file__))
    open(os.path.join(d, "randomised.bz2"), "wb").write(bytes(s))
    open(os.path.join(d, "randomised.out"), "wb").write(X)
    print("ok", len(s), "bytes, seed", seed)


if __name__ == "__main__":
    main()
