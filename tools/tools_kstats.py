"""Per-kernel ms per step from a rocprofv3 kernel_trace.csv (templates split by grid size):
python tools_kstats.py <trace.csv> [steps]"""
import collections
import csv
import sys

steps = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
agg = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].split("(")[0].split("::")[-1]
    if "bsort" in n:
        n = f"{n}<{r['Grid_Size_X']}>"
    agg[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 / steps
for k, v in sorted(agg.items(), key=lambda x: -x[1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 18]:
    print(f"{k:40s} {v:8.2f}")
print("total", round(sum(agg.values()), 2))
