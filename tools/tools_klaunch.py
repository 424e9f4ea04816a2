"""Per-launch durations (ms) of chosen kernels in the last step of a kernel trace:
tools_klaunch.py <trace.csv> k_name [k_name ...]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for name in sys.argv[2:]:
    ds = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in rows
          if r['Kernel_Name'].split('(')[0].split('<')[0].endswith(name)]
    n = len(ds) // 2
    print(f"{name:16s} {len(ds):3d} sum={sum(ds[n:]):7.2f} " + ' '.join('%.2f' % x for x in ds[n:][:30]))
