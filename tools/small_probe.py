"""Small-call timings (development tool): ms per bzg_compress_device call on the first
100 MB and 125 MB of the bench text (best of 8 warm calls each), with the stage split."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import bzip2_amd as B  # noqa: E402
from tests import datagen  # noqa: E402


def main():
    n_max = 125_000_000
    d = torch.frombuffer(bytearray(datagen.text(n_max, bench.rank_seed(0))), dtype=torch.uint8).to("cuda")
    cap = B.bound(n_max)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    res = []
    for n in (100_000_000, 125_000_000):
        best, st = 1e9, None
        for i in range(10):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            B.compress_device(d.data_ptr(), n, 9, out.data_ptr(), cap, stream_ptr=sp)
            torch.cuda.synchronize()
            ms = 1e3 * (time.perf_counter() - t0)
            if i >= 2 and ms < best:
                best, st = ms, B.last_stats()
        res.append(f"{n // 1_000_000}MB {best:.3f} ms {n / best / 1e3:.0f} MB/s " +
                   str({k: round(st[k + '_ms'], 3) for k in ('rle1', 'bwt', 'mtf', 'code')}))
    print(" | ".join(res), flush=True)


if __name__ == "__main__":
    main()
