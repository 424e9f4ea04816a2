import ctypes, os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np
import bzip2_amd as B
from tests import datagen
data = datagen.text(1_000_000_000, 0x5EED0001)
src = np.frombuffer(data, dtype=np.uint8)
cap = B.bound(len(data))
dst = np.empty(cap, dtype=np.uint8)
L = B.lib()
for it in range(3):
    dl = ctypes.c_uint(cap)
    t = time.perf_counter()
    rc = L.BZ2_bzBuffToBuffCompress(dst.ctypes.data, ctypes.byref(dl), src.ctypes.data, len(data), 9, 0, 30)
    print("h2h", it, rc, round((time.perf_counter() - t) * 1e3, 2), "ms", flush=True)
