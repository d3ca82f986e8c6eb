"""Per-step kernel time breakdown from a rocprofv3 results .db (tuning tool; the .db is rocprofv3's
default output format on this image).  usage: python tools/prof_db_summary.py DIR_OR_DB STEPS [TOP] [--csv OUT]"""
import csv
import glob
import os
import sqlite3
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
path, steps = args[0], float(args[1])
top = int(args[2]) if len(args) > 2 else 25
db = path if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "name" if "name" in cols else "kernel_name"
rows = list(c.execute(f"select {name_col}, count(*), sum(end - start), avg(end - start), min(end - start), "
                      f"max(end - start) from kernels group by {name_col} order by 3 desc"))
tot = sum(r[2] for r in rows)
print(f"total {tot / 1e6:.2f} ms over {steps:.0f} steps -> {tot / 1e3 / steps:.1f} us/step")
for n, cnt, s, a, mn, mx in rows[:top]:
    short = n.replace("void mmt::", "").replace("mmt::", "").split("(")[0][:70]
    print(f"{s / 1e3 / steps:9.1f} us/step {100 * s / tot:6.2f}%  calls/step {cnt / steps:5.1f}  avg {a / 1e3:7.1f} us  {short}")
if "--csv" in sys.argv:
    out = sys.argv[sys.argv.index("--csv") + 1]
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for n, cnt, s, a, mn, mx in rows:
            w.writerow([n, cnt, s, a, 100 * s / tot, mn, mx])
