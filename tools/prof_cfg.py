"""One compression workload for kernel tracing: python tools/prof_cfg.py <text|random|single> [bytes] [steps]

text: tests/datagen.py text; random: seeded PRNG bytes (BASELINE config 5); single: one repeated
byte (config 4).  The input is generated on the device and compressed `steps` times at -9 with
the first launch as warm-up; run under rocprofv3 with BZG_ONE_STREAM=1 for per-kernel times.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bzip2_amd as B  # noqa: E402


def main():
    kind = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000_000
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    if kind == "random":
        g = torch.Generator(device="cuda").manual_seed(0x5EED0005)
        d = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g)
    elif kind == "single":
        d = torch.full((n,), 0x61, dtype=torch.uint8, device="cuda")
    else:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
        import datagen
        d = torch.frombuffer(bytearray(datagen.text(n, 0x5EED0001)), dtype=torch.uint8).to("cuda")
    cap = B.bound(n)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    for s in range(steps):
        t = time.perf_counter()
        nb, _, _ = B.compress_device(d.data_ptr(), n, 9, out.data_ptr(), cap)
        torch.cuda.synchronize()
        print(f"step {s}: {(time.perf_counter() - t) * 1e3:.2f} ms, {nb} B, stages {B.last_stats()}", flush=True)


if __name__ == "__main__":
    main()
