"""Top kernels of a rocprofv3 kernel_stats.csv (ms per step, assuming 2 steps traced):
python tools_kstat_top.py <csv> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print(" | ".join(f"{r['Name'].split('(')[0].split('::')[-1][:14]} {float(r['TotalDurationNs']) / 2e6:.2f}" for r in rows[:n]))
