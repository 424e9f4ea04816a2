"""Times the GPU Huffman code-length routine (k_code_lengths_test, the same device code as
k_huff) on synthetic frequency tables, at several table counts, to separate one heap's latency
from throughput (development tool; run under rocprofv3 --kernel-trace --stats).

usage: python tools/huff_probe.py   (prints one line per case; kernel times come from rocprof)
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bzip2_amd as B  # noqa: E402


def tables(kind, n, seed=1):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        if kind == "prng":  # config 5: 258 symbols of near-equal counts
            out.append([int(x) for x in rng.poisson(580, 258)])
        else:  # text: a Zipf-like head, a long tail of zeros (weight 1 ties)
            a = int(rng.integers(60, 258))
            f = (20000.0 / np.arange(1, a + 1) ** 1.3).astype(np.int64)
            f[rng.random(a) < 0.3] = 0
            out.append([int(x) for x in f])
    return out


def main():
    rng = np.random.default_rng(7)
    for a in (8, 32, 64, 128, 258):  # latency against the alphabet size (no rescale: near-equal counts)
        t = [[int(x) for x in rng.poisson(580, a)] for _ in range(48)]
        B.code_lengths(t)
        B.code_lengths(t)
        print(f"alpha {a}: 48 tables", flush=True)
    for kind in ("prng", "text"):
        for n in (48, 480, 4800):
            t = tables(kind, n)
            B.code_lengths(t)  # warm
            t0 = time.perf_counter()
            B.code_lengths(t)
            print(f"{kind} {n} tables: host call {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)


if __name__ == "__main__":
    main()
