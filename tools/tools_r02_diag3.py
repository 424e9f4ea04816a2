"""Diagnostic 3: BWT of every block of the 400 MB long-repeat stream, three runs of the whole
batch: run-to-run differences and differences against the reference blocksort."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

import bench  # noqa: E402
from tests import datagen, oracles as O  # noqa: E402
from tests.test_gpu import gpu_bwt, gpu_rle1  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 400_000_000
d = torch.frombuffer(bytearray(datagen.text(n, 0x5EED0007)), dtype=torch.uint8).to("cuda")
bench.add_repeats(d, 0.25)
data = d.cpu().numpy().tobytes()
blocks, offs, crcs = gpu_rle1(data, 9)
nb = len(offs) - 1
runs = [gpu_bwt(blocks, offs) for _ in range(3)]
for i in (1, 2):
    diff = [k for k in range(nb) if runs[i][0][offs[k]:offs[k + 1]] != runs[0][0][offs[k]:offs[k + 1]]
            or runs[i][1][k] != runs[0][1][k]]
    print(f"run {i} vs run 0: {len(diff)} blocks differ {diff[:10]}", flush=True)
t = time.time()
bad = []
for k in range(nb):
    blk = blocks[offs[k]:offs[k + 1]]
    ref = ctypes.create_string_buffer(len(blk))
    ro = O.ref().ref_blocksort(blk, len(blk), ref)
    got = runs[0][0][offs[k]:offs[k + 1]]
    if got != ref.raw or runs[0][1][k] != ro:
        dp = [i for i in range(len(blk)) if got[i] != ref.raw[i]]
        bad.append(k)
        if len(bad) <= 5:
            print(f"block {k}: len {len(blk)} ndiff {len(dp)} first {dp[:8]} origptr {runs[0][1][k]} vs {ro}", flush=True)
print(f"blocks differing from the reference: {len(bad)} of {nb} {bad[:20]} ({time.time() - t:.0f}s)", flush=True)
