"""Host-to-host components on this box (development tool): pageable H2D of 1e9 B, the
device-resident call, and BZ2_bzBuffToBuffCompress (BZG_H2H_DEBUG=1 prints its timeline)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bzip2_amd as B  # noqa: E402
from tests import datagen  # noqa: E402

data = datagen.text(1_000_000_000, 0x5EED0001)
src = np.frombuffer(data, dtype=np.uint8)
d = torch.empty(len(data), dtype=torch.uint8, device="cuda")
for i in range(3):
    torch.cuda.synchronize()
    t = time.perf_counter()
    d.copy_(torch.from_numpy(src))
    torch.cuda.synchronize()
    print(f"h2d pageable 1e9 B: {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
cap = B.bound(len(data))
out = torch.empty(cap, dtype=torch.uint8, device="cuda")
sp = torch.cuda.current_stream().cuda_stream
for i in range(3):
    torch.cuda.synchronize()
    t = time.perf_counter()
    nb, _, _ = B.compress_device(d.data_ptr(), len(data), 9, out.data_ptr(), cap, stream_ptr=sp)
    torch.cuda.synchronize()
    print(f"device call: {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
host = np.empty(nb, dtype=np.uint8)
for i in range(3):
    t = time.perf_counter()
    host[:] = out[:nb].cpu().numpy()
    print(f"d2h {nb} B: {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
dst = np.empty(cap, dtype=np.uint8)
L = B.lib()
for i in range(4):
    dl = ctypes.c_uint(cap)
    t = time.perf_counter()
    rc = L.BZ2_bzBuffToBuffCompress(dst.ctypes.data, ctypes.byref(dl), src.ctypes.data, len(data), 9, 0, 30)
    print("h2h", i, rc, f"{1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
