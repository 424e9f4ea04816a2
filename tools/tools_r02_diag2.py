"""Diagnostic 2: repeatability of the block-382 mismatch inside an 80-block batch."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench  # noqa: E402
from tests import datagen, oracles as O  # noqa: E402
from tests.test_gpu import gpu_bwt, gpu_rle1  # noqa: E402

n = 400_000_000
d = torch.frombuffer(bytearray(datagen.text(n, 0x5EED0007)), dtype=torch.uint8).to("cuda")
bench.add_repeats(d, 0.25)
data = d.cpu().numpy().tobytes()
blocks, offs, crcs = gpu_rle1(data, 9)
k = 382
blk = blocks[offs[k]:offs[k + 1]]
ref_bwt = ctypes.create_string_buffer(len(blk))
ro = O.ref().ref_blocksort(blk, len(blk), ref_bwt)
for (lo, hi) in [(k - 40, k + 40), (k - 40, k + 40), (k - 40, k + 40), (k - 1, k + 1), (k - 10, k + 1), (k, k + 10),
                 (k - 20, k + 20), (0, len(offs) - 1)]:
    lo, hi = max(0, lo), min(len(offs) - 1, hi)
    sub = blocks[offs[lo]:offs[hi]]
    so = [x - offs[lo] for x in offs[lo:hi + 1]]
    bw, op = gpu_bwt(sub, so)
    j = k - lo
    got = bw[so[j]:so[j + 1]]
    dp = [i for i in range(len(blk)) if got[i] != ref_bwt.raw[i]]
    bad_blocks = []
    for b in range(lo, hi):
        rb = ctypes.create_string_buffer(offs[b + 1] - offs[b])
        if b != k and b % 7 == 0:
            O.ref().ref_blocksort(blocks[offs[b]:offs[b + 1]], offs[b + 1] - offs[b], rb)
            if bw[so[b - lo]:so[b - lo + 1]] != rb.raw:
                bad_blocks.append(b)
    print(f"batch [{lo},{hi}) block {k}: equal {not dp} ndiff {len(dp)} first {dp[:8]} origptr {op[j]} vs {ro} "
          f"other bad (sampled) {bad_blocks}", flush=True)
