"""Summarise a rocprofv3 kernel_stats.csv: python tools_stats.py <csv> [steps]"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:22]:
    print(f'{r["Name"][:34]:34s} calls={int(r["Calls"])/steps:7.1f} ms/step={float(r["TotalDurationNs"])/1e6/steps:8.2f} '
          f'avg={float(r["AverageNs"])/1e3:9.1f}us {100*float(r["TotalDurationNs"])/tot:5.1f}%')
print("total kernel ms/step", tot / 1e6 / steps)
