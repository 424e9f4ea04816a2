"""Per-kernel sums of PMC counters from tools_pmc.sh output: python tools_pmcsum.py <dir>"""
import collections
import csv
import glob
import re
import sys


def short(name):
    m = re.search(r"::(k_\w+)", name)
    return m.group(1) if m else name[:30]


agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        if k == "k_bsort":
            k += "<%s>" % r["Grid_Size"]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
names = sorted({c for k in agg.values() for c in k})
print(f'{"kernel":22s} ' + " ".join(f"{n[3:17]:>14s}" for n in names))
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1].values()))[:24]:
    print(f"{k:22s} " + " ".join(f"{v.get(n, 0):14.4g}" for n in names))
