"""Split the rocprofv3 kernel trace's residual-epilogue f16x3 GEMM launches into proj and fc2 (tuning tool).

With the two-stream halves off, each ViT block launches proj then fc2 on the same kernel and the same grid, so
the trace tells them apart by order only. Prints both means, to set against the bench line's per-class probe.
usage: python tools/prof_split_resid.py <run_kernel_trace.csv>
"""
import csv
import statistics
import sys

NAMES = ("gemm_kernel<128, 128, 4, 2, 2, 0, true, 2, 64>", "gemm128w_kernel<2>")   # (the 128 x 256 tile: the 320-token layers)
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
for NAME in NAMES:
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows if NAME in r["Kernel_Name"]]
    if not d:
        continue
    if len(d) % 2:
        raise SystemExit(f"expected proj / fc2 pairs of {NAME}, found {len(d)} launches")
    print(f"{len(d)} launches of {NAME}: proj {statistics.mean(d[0::2]):.2f} us, fc2 {statistics.mean(d[1::2]):.2f} us "
          f"(mean per launch, {len(d) // 2} each)")
