"""Summarise rocprofv3 --pmc CSVs: per kernel (name filter), mean counter value per dispatch."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "mmt::"
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].replace("void mmt::", "").split("(mmt::")[0][:70]
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in vals.items():
    print(name)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} n={len(v):4d} mean={sum(v) / len(v):16.1f}")
