"""Decode profiling driver: compress N bytes of the bench text once, then decode it `reps`
times device-resident (run under rocprofv3 --kernel-trace --stats)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

import bzip2_amd as B  # noqa: E402
from tests import datagen  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
kind = sys.argv[3] if len(sys.argv) > 3 else "text"
data = datagen.text(n, 0x5EED0001) if kind == "text" else datagen.random_bytes(n, 5)
d = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
cap = B.bound(n)
o = torch.empty(cap, dtype=torch.uint8, device="cuda")
nb, _, _ = B.compress_device(d.data_ptr(), n, 9, o.data_ptr(), cap)
dd = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
for r in range(reps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    rc, got = B.decompress_device(o.data_ptr(), nb, dd.data_ptr(), n + 64)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"rep {r}: rc {rc} got {got} {dt * 1e3:.1f} ms {n / dt / 1e6:.0f} MB/s", B.last_decode_stats(), flush=True)
assert torch.equal(dd[:n], d)
print("decode ok")
