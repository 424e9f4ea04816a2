"""HBM traffic per step from the two PMC passes of tools_r01_gpu.sh (FETCH_SIZE, WRITE_SIZE;
rocprofv3 reports both in KB).  Correction per MI355X_MICROARCH.md (HBM section): on gfx950
FETCH_SIZE counts half the bytes of wide streaming reads, so the corrected read figure is
2 x FETCH_SIZE; WRITE_SIZE is taken as is.  Random 4-byte gathers (the sort kernels) are not
calibrated by that rule, so the uncorrected figure is kept beside it as a lower bound.
usage: python tools_traffic.py <pmc_dir> <bench.json> <out.json>"""
import collections
import csv
import json
import sys


def per_kernel(path):
    agg = collections.Counter()
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)", "").split("(")[0].split("::")[-1]
        agg[name.split("<")[0]] += float(r["Counter_Value"]) * 1024.0  # KB -> B
    return agg


d, bj, out = sys.argv[1:4]
fetch = per_kernel(d + "/p1/run_counter_collection.csv")
write = per_kernel(d + "/p2/run_counter_collection.csv")
bench = json.loads(open(bj).read().strip().splitlines()[-1])
ms = bench["ms_per_step"]
tot_f, tot_w = sum(fetch.values()), sum(write.values())
corr = 2.0 * tot_f + tot_w
kern = {k: {"fetch_raw_B": fetch[k], "write_B": write[k]} for k in sorted(set(fetch) | set(write),
                                                                          key=lambda k: -(fetch[k] + write[k]))}
res = {
    "workload": bench["config"]["workload"],
    "bytes_per_step": bench["config"]["bytes_per_gpu"],
    "ms_per_step_bench": ms,
    "fetch_raw_B": tot_f, "write_B": tot_w,
    "traffic_B_per_step": corr, "traffic_lower_B_per_step": tot_f + tot_w,
    "traffic_GBps": corr / (ms / 1e3) / 1e9,
    "correction": "2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM section); lower = raw sum",
    "per_kernel": kern,
}
json.dump(res, open(out, "w"), indent=1)
print(f"fetch {tot_f/1e9:.1f} GB raw, write {tot_w/1e9:.1f} GB, corrected {corr/1e9:.1f} GB per step "
      f"= {res['traffic_GBps']:.0f} GB/s over {ms} ms")
for k, v in list(kern.items())[:12]:
    print(f"  {k:24s} fetch {v['fetch_raw_B']/1e9:7.2f} GB  write {v['write_B']/1e9:7.2f} GB")
