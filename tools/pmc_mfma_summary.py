"""Per-kernel means of the tools/pmc_mfma.sh counters (tuning tool)."""
import csv
import glob
import sys
from collections import defaultdict

v = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mmt::" in r["Kernel_Name"]:
            k = r["Kernel_Name"].replace("void mmt::", "").split("(")[0][:60]
            v[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(v.items()):
    m = {c: sum(x) / len(x) for c, x in cs.items()}
    line = f"{k:60s} " + " ".join(f"{c}={m[c]:.4g}" for c in sorted(m))
    if "GRBM_GUI_ACTIVE" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m and m["GRBM_GUI_ACTIVE"] > 0:
        line += f"  mfma_busy/(gui/8*1024)={m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}"
    print(line)
