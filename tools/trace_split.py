"""Split a rocprofv3 kernel trace into compression steps and the setup before them.

usage: python tools/trace_split.py <run_kernel_trace.csv> [first-kernel-of-a-step]

A step starts at each launch of the pipeline's first kernel (RLE1's count pass); everything
before the first step (input upload through pageable staging buffers, warm-up allocations)
is reported separately, so blit kernels such as __amd_rocclr_copyBuffer are charged to the
steps only when they run inside one.
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "k_rle_count"
    rows = list(csv.DictReader(open(path)))
    for r in rows:  # full demangled names (no -T): "void bzg::(anonymous namespace)::k_x<...>(args)"
        n = r["Kernel_Name"]
        if n.startswith("void "):
            n = n[5:]
        n = n.replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].split("::")[-1]
        r["Kernel_Name"] = n
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [int(r["Start_Timestamp"]) for r in rows if r["Kernel_Name"].startswith(first)]
    if not starts:
        first = "k_run_starts"
        starts = [int(r["Start_Timestamp"]) for r in rows if r["Kernel_Name"].startswith(first)]
    if not starts:
        sys.exit(f"no launch of {first} in the trace")
    setup = collections.Counter()
    inside = collections.Counter()
    calls_in = collections.Counter()
    for r in rows:
        name = r["Kernel_Name"].split("(")[0][:48]
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if int(r["Start_Timestamp"]) < starts[0]:
            setup[name] += dur
        else:
            inside[name] += dur
            calls_in[name] += 1
    ns = len(starts)
    print(f"steps: {ns} (launches of {first})")
    print("setup before the first step (ms):")
    for k, v in setup.most_common(6):
        print(f"  {k:48s} {v / 1e6:9.2f}")
    print("per step (ms, calls):")
    for k, v in inside.most_common(40):
        print(f"  {k:48s} {v / 1e6 / ns:9.3f} {calls_in[k] / ns:8.1f}")


if __name__ == "__main__":
    main()
