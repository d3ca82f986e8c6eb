"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV (tuning tool, not a test).

Takes the last `steps` occurrences of the step's first kernel (crop_kernel) as step boundaries and
reports, per step: busy time (union of kernel intervals), idle gaps between consecutive kernels, and
the time per kernel class.  usage: python tools/trace_gaps.py <kernel_trace.csv> [steps]
"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = [r for r in csv.DictReader(open(path))]
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
starts = [i for i, e in enumerate(ev) if "crop_kernel" in e[2]]
if len(starts) < steps + 1:
    sys.exit(f"only {len(starts)} crop_kernel launches")
sel = starts[-(steps + 1):]
per = defaultdict(float)
busy = gaps = span = 0.0
ngaps = 0
for a, b in zip(sel[:-1], sel[1:]):
    seg = ev[a:b]
    span += (ev[b][0] - seg[0][0]) / 1e3
    end = seg[0][0]
    for s, e, n in seg:
        if s > end:
            gaps += (s - end) / 1e3
            ngaps += 1
        busy += max(0, e - max(s, end)) / 1e3
        end = max(end, e)
        name = n.replace("void mmt::", "").replace("mmt::", "").split("(")[0]
        per[name] += (e - s) / 1e3
print(f"{steps} steps: span {span / steps:.1f} us/step, busy {busy / steps:.1f}, idle gaps {gaps / steps:.1f} "
      f"({ngaps / steps:.0f} gaps/step, {len(ev[sel[0]:sel[-1]]) / steps:.0f} kernels/step)")
for name, t in sorted(per.items(), key=lambda kv: -kv[1]):
    print(f"  {t / steps:8.1f} us/step  {name[:90]}")
