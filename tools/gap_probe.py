"""Where a small compress call's fixed cost goes (development tool): compresses N bytes of the
bench text on the device a few times; run under rocprofv3 --kernel-trace, then
`python tools/gap_probe.py --report <kernel_trace.csv>` lists, for the last call, the wall time,
the kernel-busy time (union of kernel intervals) and the largest idle gaps with the kernels
around them.

usage: python tools/gap_probe.py [bytes]            (on the GPU box, under rocprofv3)
       python tools/gap_probe.py --report <csv>     (anywhere)
"""
import csv
import os
import re
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(n):
    import torch

    import bench
    import bzip2_amd as B
    from tests import datagen

    d = torch.frombuffer(bytearray(datagen.text(n, bench.rank_seed(0))), dtype=torch.uint8).to("cuda")
    cap = B.bound(n)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    sp = torch.cuda.current_stream().cuda_stream
    for i in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        B.compress_device(d.data_ptr(), n, 9, out.data_ptr(), cap, stream_ptr=sp)
        torch.cuda.synchronize()
        print(f"call {i}: {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)


def report(path):
    rows = list(csv.DictReader(open(path)))
    nm = lambda r: re.sub(r"^(void )?bzg::\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0][:40]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm(r)) for r in rows)
    starts = [i for i, k in enumerate(ks) if k[2].startswith("k_rle_count")]
    last = ks[starts[-1]:]
    t0, t1 = last[0][0], max(e for _, e, _ in last)
    busy, cur_s, cur_e, gaps = 0, last[0][0], last[0][1], []
    prev = last[0]
    for s, e, n in last[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev[2], n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        if e >= cur_e:
            prev = (s, e, n)
    busy += cur_e - cur_s
    print(f"last call: first kernel to last end {1e-6 * (t1 - t0):.3f} ms, kernels busy {1e-6 * busy:.3f} ms, "
          f"{len(last)} kernels, {len(gaps)} gaps, idle {1e-6 * sum(g for g, _, _ in gaps):.3f} ms")
    for g, a, b in sorted(gaps, reverse=True)[:25]:
        print(f"  {g / 1e3:8.1f} us  after {a:40s} before {b}")
    tot = {}
    for s, e, n in last:
        c, t = tot.get(n, (0, 0))
        tot[n] = (c + 1, t + e - s)
    print("per kernel in the last call (us, launches):")
    for n, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"  {n:40s} {t / 1e3:9.1f} {c:5d}")


if __name__ == "__main__":
    if sys.argv[1:2] == ["--report"]:
        report(sys.argv[2])
    else:
        run(int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000)
