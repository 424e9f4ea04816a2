"""Per-kernel sums of PMC counters from tools_r02_pmc.sh output: L2 hit rate, HBM-side bytes
(FETCH_SIZE / WRITE_SIZE, KB counters -> GB) and SQ instruction / wait counters per kernel.
python tools_pmcsum.py <dir> [top]"""
import collections
import csv
import glob
import re
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"::(k_\w+)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"].split("(")[0][:26]
        if k == "k_bsort":
            k += "<%s>" % r["Grid_Size"]
        v = float(r["Counter_Value"])
        if r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
            v *= 1024.0
        agg[k][r["Counter_Name"]] += v
top = int(sys.argv[2]) if len(sys.argv) > 2 else 24
cols = ["FETCH", "WRITE", "L2hit", "VALU_M", "LDS_M", "VMEM_M", "waveGcyc", "wait%", "ldsconf", "waitLDS%", "park%", "act%",
        "actVALU%", "actLDS%", "actVMEM%"]
print(f'{"kernel":26s} ' + " ".join(f"{c:>8s}" for c in cols))
key = "SQ_WAVE_CYCLES" if any("SQ_WAVE_CYCLES" in v for v in agg.values()) else "FETCH_SIZE"
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get(key, 0))[:top]:
    h, mi = v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0)
    wc = v.get("SQ_WAVE_CYCLES", 0) or 1
    vals = [v.get("FETCH_SIZE", 0) / 1e9, v.get("WRITE_SIZE", 0) / 1e9, h / (h + mi) if h + mi else 0,
            v.get("SQ_INSTS_VALU", 0) / 1e6, v.get("SQ_INSTS_LDS", 0) / 1e6, v.get("SQ_INSTS_VMEM", 0) / 1e6,
            v.get("SQ_WAVE_CYCLES", 0) / 1e9, v.get("SQ_WAIT_INST_ANY", 0) / wc, v.get("SQ_LDS_BANK_CONFLICT", 0) / 1e6,
            v.get("SQ_WAIT_INST_LDS", 0) / wc, v.get("SQ_WAIT_ANY", 0) / wc, v.get("SQ_ACTIVE_INST_ANY", 0) / wc,
            v.get("SQ_ACTIVE_INST_VALU", 0) / wc, v.get("SQ_ACTIVE_INST_LDS", 0) / wc, v.get("SQ_ACTIVE_INST_VMEM", 0) / wc]
    print(f"{k:26s} " + " ".join(f"{x:8.3f}" for x in vals))
