"""Diagnostic: which blocks of the 400 MB long-repeat stream differ from the reference, and does
the first one reproduce alone through bzg_stage_bwt?  Writes gpurun_out/diag/."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench  # noqa: E402
import bzip2_amd as B  # noqa: E402
from tests import datagen, oracles as O  # noqa: E402
from tests.test_gpu import gpu_bwt, gpu_rle1  # noqa: E402

out_dir = "gpurun_out/diag"
os.makedirs(out_dir, exist_ok=True)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 400_000_000
d = torch.frombuffer(bytearray(datagen.text(n, 0x5EED0007)), dtype=torch.uint8).to("cuda")
bench.add_repeats(d, 0.25)
data = d.cpu().numpy().tobytes()
cap = B.bound(n)
out = torch.empty(cap, dtype=torch.uint8, device="cuda")
nb, _, _ = B.compress_device(d.data_ptr(), n, 9, out.data_ptr(), cap)
torch.cuda.synchronize()
g = out[:nb].clone()
r = O.ref_compress(data, 9)
rt = torch.frombuffer(bytearray(r), dtype=torch.uint8).to("cuda")
mg = [o for o, k in B.find_magics(g.data_ptr(), g.numel())]
mr = [o for o, k in B.find_magics(rt.data_ptr(), rt.numel())]
print("stream bytes", g.numel(), len(r), "magics", len(mg), len(mr), flush=True)
gb = np.unpackbits(g.cpu().numpy())
rb = np.unpackbits(np.frombuffer(r, np.uint8))
bad = []
for i in range(min(len(mg), len(mr)) - 1):
    a = gb[mg[i]:mg[i + 1]]
    b = rb[mr[i]:mr[i + 1]]
    if len(a) != len(b) or not np.array_equal(a, b):
        bad.append(i)
print("differing blocks", len(bad), bad[:20], flush=True)
if bad:
    blocks, offs, crcs = gpu_rle1(data, 9)
    k = bad[0]
    blk = blocks[offs[k]:offs[k + 1]]
    open(f"{out_dir}/block{k}.bin", "wb").write(blk)
    bw, op = gpu_bwt(blk, [0, len(blk)])
    ref_bwt = ctypes.create_string_buffer(len(blk))
    ro = O.ref().ref_blocksort(blk, len(blk), ref_bwt)
    print("block", k, "len", len(blk), "alone: bwt equal", bw == ref_bwt.raw, "origptr", op[0], ro, flush=True)
    # the block inside its batch neighbourhood
    lo, hi = max(0, k - 40), min(len(offs) - 1, k + 40)
    sub = blocks[offs[lo]:offs[hi]]
    so = [x - offs[lo] for x in offs[lo:hi + 1]]
    bw2, op2 = gpu_bwt(sub, so)
    j = k - lo
    print("in 80-block batch: bwt equal", bw2[so[j]:so[j + 1]] == ref_bwt.raw, "origptr", op2[j], flush=True)
    bw3, op3 = gpu_bwt(blocks, offs)
    print("in full batch: bwt equal", bw3[offs[k]:offs[k + 1]] == ref_bwt.raw, "origptr", op3[k], flush=True)
    diffpos = [i for i in range(len(blk)) if bw3[offs[k] + i] != ref_bwt.raw[i]]
    print("diff positions", len(diffpos), diffpos[:20], flush=True)
