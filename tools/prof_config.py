"""One BASELINE config on the device for profiling (development tool):
python tools/prof_config.py single|random|repeat|text [steps] [decode]
single: 4 GiB of byte 0x61 (config 4); random: 4 GiB of PRNG bytes (config 5); repeat: 1e9 B
of the bench text with 25% long repeats.  Each step is one bzg_compress_device call at -9."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import bzip2_amd as B  # noqa: E402
from tests import datagen  # noqa: E402


def main():
    kind = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    if kind == "single":
        d = torch.full((1 << 32,), 0x61, dtype=torch.uint8, device="cuda")
    elif kind == "random":
        g = torch.Generator(device="cuda")
        g.manual_seed(0x5EED0005)
        d = torch.randint(0, 256, (1 << 32,), dtype=torch.uint8, device="cuda", generator=g)
    else:
        d = torch.frombuffer(bytearray(datagen.text(1_000_000_000, bench.rank_seed(0))), dtype=torch.uint8).to("cuda")
        if kind == "repeat":
            bench.add_repeats(d, 0.25)
    n = d.numel()
    cap = B.bound(n)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    ms, nb, st = bench.time_device(d, n, 9, out, cap, steps=steps)
    if len(sys.argv) > 3 and sys.argv[3] == "decode":  # then decode the stream `steps` times
        dec = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        sp = torch.cuda.current_stream().cuda_stream
        for _ in range(steps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rc, got = B.decompress_device(out.data_ptr(), nb, dec.data_ptr(), n + 64, stream_ptr=sp)
            torch.cuda.synchronize()
            print("decode", rc, got, f"{1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
    print(kind, n, f"{ms:.3f} ms", f"{n / ms / 1e3:.1f} MB/s", {k: round(st[k + '_ms'], 3) for k in ("rle1", "bwt", "mtf", "code")},
          flush=True)


if __name__ == "__main__":
    t = time.time()
    main()
    print(f"{time.time() - t:.1f} s")
