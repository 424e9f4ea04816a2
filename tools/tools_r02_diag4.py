"""Diagnostic 4: the nondeterministic long-repeat mismatch.  Repeats the whole-batch BWT of the
400 MB long-repeat stream; for every block that differs from the reference, the rotations at the
differing sorted positions and their common prefix length (cyclic suffix array by numpy
prefix doubling)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

import bench  # noqa: E402
from tests import datagen, oracles as O  # noqa: E402
from tests.test_gpu import gpu_bwt, gpu_rle1  # noqa: E402


def cyc_sa(b):
    t = np.frombuffer(b, np.uint8).astype(np.int64)
    n = len(t)
    rank = t.copy()
    h = 1
    while True:
        key = rank * (n + 1) + rank[(np.arange(n) + h) % n]
        sa = np.argsort(key, kind="stable")
        ks = key[sa]
        nr = np.empty(n, np.int64)
        nr[sa] = np.concatenate([[0], np.cumsum(ks[1:] != ks[:-1])])
        rank = nr
        if rank.max() == n - 1 or h >= n:
            return sa
        h *= 2


def lcp(b, x, y, cap=1 << 20):
    n = len(b)
    k = 0
    while k < min(n, cap) and b[(x + k) % n] == b[(y + k) % n]:
        k += 1
    return k


if __name__ == "__main__":
    n = 400_000_000
    d = torch.frombuffer(bytearray(datagen.text(n, 0x5EED0007)), dtype=torch.uint8).to("cuda")
    bench.add_repeats(d, 0.25)
    data = d.cpu().numpy().tobytes()
    blocks, offs, crcs = gpu_rle1(data, 9)
    nb = len(offs) - 1
    refs = {}
    for rep in range(int(os.environ.get("REPS", "4"))):
        bw, op = gpu_bwt(blocks, offs)
        bad = []
        for k in range(nb):
            blk = blocks[offs[k]:offs[k + 1]]
            if k not in refs:
                ref = ctypes.create_string_buffer(len(blk))
                ro = O.ref().ref_blocksort(blk, len(blk), ref)
                refs[k] = (ref.raw, ro)
            if bw[offs[k]:offs[k + 1]] != refs[k][0] or op[k] != refs[k][1]:
                bad.append(k)
        print(f"rep {rep}: bad blocks {bad}", flush=True)
        for k in bad[:2]:
            blk = blocks[offs[k]:offs[k + 1]]
            got = bw[offs[k]:offs[k + 1]]
            dp = [i for i in range(len(blk)) if got[i] != refs[k][0][i]]
            sa = cyc_sa(blk)
            for p in dp[:4]:
                a, b = int(sa[p]), int(sa[p + 1]) if p + 1 < len(blk) else -1
                print(f"  block {k} pos {p}: rot {a} next {b} lcp(p,p+1) {lcp(blk, a, b) if b >= 0 else -1}"
                      f" lcp(p-1,p) {lcp(blk, int(sa[p - 1]), a)}", flush=True)
