"""Per-step kernel time breakdown from a rocprofv3 --stats kernel_stats.csv (tuning tool)."""
import csv
import sys

path, steps = sys.argv[1], float(sys.argv[2])
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.2f} ms over {steps:.0f} steps -> {tot / 1e3 / steps:.1f} us/step")
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    name = r["Name"].replace("void mmt::", "").replace("mmt::", "").split("(")[0][:60]
    print(f"{float(r['TotalDurationNs']) / 1e3 / steps:9.1f} us/step {float(r['Percentage']):6.2f}%  "
          f"calls/step {float(r['Calls']) / steps:5.1f}  avg {float(r['AverageNs']) / 1e3:7.1f} us  {name}")
