"""Split the rocprofv3 kernel trace's residual-epilogue f16x3 GEMM launches into proj and fc2 (tuning tool).

With the two-stream halves off, each ViT block launches proj then fc2 (EPI_RESID_F32 = 2 on whichever tile the
dispatch picks: gemm_kernel<.., 2, ..>, gemm128w_kernel<2>, gemm256s_kernel<2, 4>), so the trace tells them apart by
order only. Prints both classes' means per kernel, to set against the bench line's per-class probe.
usage: python tools/prof_split_resid.py <run_kernel_trace.csv>
"""
import csv
import re
import statistics
import sys
from collections import defaultdict


def resid(name):
    m = re.search(r"(gemm\w*_kernel)<([^>]*)>", name)
    if not m:
        return False
    args = [a.strip() for a in m.group(2).split(",")]
    if m.group(1) == "gemm_kernel":
        return len(args) > 4 and args[4] == "2"
    return args[0] == "2"


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
d = [(re.search(r"gemm\w*_kernel<[^>]*>", r["Kernel_Name"]).group(0),
      (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000) for r in rows if resid(r["Kernel_Name"])]
if not d or len(d) % 2:
    raise SystemExit(f"expected proj / fc2 pairs of residual GEMMs, found {len(d)} launches")
cls = defaultdict(list)
for i, (k, us) in enumerate(d):
    cls[("proj" if i % 2 == 0 else "fc2", k)].append(us)
for c in ("proj", "fc2"):
    allc = [u for (cc, k), v in cls.items() if cc == c for u in v]
    parts = ", ".join(f"{k} {statistics.mean(v):.2f} us x {len(v)}" for (cc, k), v in sorted(cls.items()) if cc == c)
    print(f"{c}: mean {statistics.mean(allc):.2f} us per launch over {len(allc)} ({parts})")
