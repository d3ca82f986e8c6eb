"""Per-step kernel time breakdown from a rocprofv3 --stats kernel_stats.csv (tuning tool).

usage: prof_summary.py kernel_stats.csv [steps|auto] [rows]
Steps default to 'auto': the number of geometry_kernel dispatches (once per mmt_track_batch launch split into stream
halves, before they fork) plus crop_kernel<true> dispatches (a one-stream launch forms its geometry in the crop, once
per launch), so every launched step -- warm-up and timed alike -- is counted once and per-step figures are exact for
runs whose launches all have one shape (--probe none)."""
import csv
import sys

path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
arg = sys.argv[2] if len(sys.argv) > 2 else "auto"
if arg == "auto":
    steps = float(sum(float(r["Calls"]) for r in rows
                      if "geometry_kernel" in r["Name"] or "crop_kernel<true>" in r["Name"]))
    if not steps:   # the mfDiMP path: one dimp_localize_kernel per tracked frame of the batch
        steps = float(sum(float(r["Calls"]) for r in rows if "dimp_localize_kernel" in r["Name"]))
else:
    steps = float(arg)
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.2f} ms over {steps:.0f} steps -> {tot / 1e3 / steps:.1f} us/step (kernel time; two-stream "
      f"halves overlap, so this can exceed the wall time of a step)")
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    name = r["Name"].replace("void mmt::", "").replace("mmt::", "").split("(")[0][:60]
    print(f"{float(r['TotalDurationNs']) / 1e3 / steps:9.1f} us/step {float(r['Percentage']):6.2f}%  "
          f"calls/step {float(r['Calls']) / steps:5.1f}  avg {float(r['AverageNs']) / 1e3:7.1f} us  {name}")
