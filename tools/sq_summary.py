"""Per-kernel SQ counter summary from a rocprofv3 --pmc counter_collection.csv:
python tools/sq_summary.py <counter_collection.csv> [top] [--tmpl] [--lds <second pass csv>]
(--tmpl: keep template arguments).  Prints per kernel: waves, VALU / LDS / VMEM-read
instructions per wave, and the split of wave cycles into active-issue, issue-stall
(WAIT_INST_ANY) and parked (WAIT_ANY) fractions; with --lds, the LDS bank-conflict cycles per
LDS-active cycle (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE) from the second counter pass."""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.Counter())
tmpl = "--tmpl" in sys.argv
sys.argv = [a for a in sys.argv if a != "--tmpl"]
lds = None
if "--lds" in sys.argv:
    i = sys.argv.index("--lds")
    lds = sys.argv[i + 1]
    del sys.argv[i:i + 2]


def name(r):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("::")[-1]
    return n if tmpl else n.split("<")[0]


for r in csv.DictReader(open(sys.argv[1])):
    agg[name(r)][r["Counter_Name"]] += float(r["Counter_Value"])
if lds:
    for r in csv.DictReader(open(lds)):
        if r["Counter_Name"] != "SQ_WAVES":
            agg[name(r)][r["Counter_Name"]] += float(r["Counter_Value"])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = sorted(agg.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"])[:top]
print(f"{'kernel':40s} {'waves':>10s} {'valu/w':>8s} {'lds/w':>7s} {'vmem/w':>7s} {'act':>5s} {'stall':>5s} {'park':>5s} {'Gcyc':>7s}"
      + (f" {'ldsconf':>7s}" if lds else ""))
for n, c in rows:
    w = max(c["SQ_WAVES"], 1)
    wc = max(c["SQ_WAVE_CYCLES"], 1)
    print(f"{n[:40]:40s} {int(w):10d} {c['SQ_INSTS_VALU']/w:8.0f} {c['SQ_INSTS_LDS']/w:7.0f} {c['SQ_INSTS_VMEM_RD']/w:7.0f} "
          f"{c['SQ_ACTIVE_INST_ANY']/wc:5.2f} {c['SQ_WAIT_INST_ANY']/wc:5.2f} {c['SQ_WAIT_ANY']/wc:5.2f} {wc/1e9:7.2f}"
          + (f" {c['SQ_LDS_BANK_CONFLICT']/max(c['SQ_LDS_IDX_ACTIVE'], 1):7.3f}" if lds else ""))
