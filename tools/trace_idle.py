"""Idle time of the GPU in the last part of a rocprofv3 --kernel-trace CSV (tuning tool, not a test): the union
of kernel intervals over the last `window_ms`, and the largest idle gaps with the kernels around them.
usage: python tools/trace_idle.py <kernel_trace.csv> [window_ms] [top]"""
import csv
import sys

path = sys.argv[1]
window = float(sys.argv[2]) if len(sys.argv) > 2 else 50.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path)))
t_end = max(e for _, e, _ in ev)
t0 = t_end - window * 1e6
ev = [x for x in ev if x[0] >= t0]
short = lambda n: n.replace("void mmt::", "").replace("mmt::", "").split("(")[0][:60]
busy, end, gaps = 0.0, ev[0][0], []
prev = ev[0][2]
for s, e, n in ev:
    if s > end:
        gaps.append(((s - end) / 1e3, short(prev), short(n)))
    busy += max(0, e - max(s, end)) / 1e3
    if e > end:
        end, prev = e, n
span = (end - ev[0][0]) / 1e3
print(f"last {window:.0f} ms: {len(ev)} kernels, busy {busy:.1f} us of {span:.1f} us ({100 * busy / span:.1f} %), "
      f"{len(gaps)} gaps, {sum(g[0] for g in gaps):.1f} us idle")
for g in sorted(gaps, reverse=True)[:top]:
    print(f"  gap {g[0]:8.1f} us  after {g[1]}  before {g[2]}")
