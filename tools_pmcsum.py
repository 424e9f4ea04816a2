"""Per-kernel sums of PMC counters from tools_r02_pmc.sh output (KB counters converted to
bytes), with the L2 hit rate when TCC_HIT/TCC_MISS were collected:
python tools_pmcsum.py <dir> [top]"""
import collections
import csv
import glob
import re
import sys


def short(name):
    m = re.search(r"::(k_\w+)", name)
    n = m.group(1) if m else name.split("(")[0][:30]
    return n


agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        v = float(r["Counter_Value"])
        if r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
            v *= 1024.0
        agg[k][r["Counter_Name"]] += v
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
print(f'{"kernel":22s} {"FETCH GB":>9s} {"WRITE GB":>9s} {"L2 hit":>7s} {"HIT+MISS G":>10s}')
for k, v in sorted(agg.items(), key=lambda kv: -(kv[1].get("FETCH_SIZE", 0) + kv[1].get("WRITE_SIZE", 0)))[:top]:
    h, m = v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0)
    hr = f"{h / (h + m):7.3f}" if h + m else "      -"
    print(f"{k:22s} {v.get('FETCH_SIZE', 0) / 1e9:9.2f} {v.get('WRITE_SIZE', 0) / 1e9:9.2f} {hr} {(h + m) / 1e9:10.3f}")
