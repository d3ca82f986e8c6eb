"""Per-launch-position durations of a rocprofv3 kernel trace (tuning tool): the k-th launch of each kernel inside a step
(e.g. the layer index of a one-launch-per-layer GEMM), averaged over the steady steps.

usage: python tools/trace_layers.py TRACE.csv MARKER_KERNEL SKIP_STEPS [NAME_FILTER ...]
A step starts at each launch of MARKER_KERNEL (crop_kernel<true> for a one-stream launch); the first SKIP_STEPS
steps and the last (partial) one are dropped."""
import collections
import csv
import gzip
import sys


def main():
    path, marker, skip = sys.argv[1], sys.argv[2], int(sys.argv[3])
    filt = sys.argv[4:]
    rows = list(csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    steps = [rows[idx[k]:idx[k + 1]] for k in range(skip, len(idx) - 1)]
    dur = collections.defaultdict(list)
    order = []
    for st in steps:
        seen = collections.Counter()
        for r in st:
            name = r["Kernel_Name"].replace("void mmt::", "").replace("mmt::", "").split("(")[0][:64]
            if filt and not any(f in name for f in filt):
                continue
            key = (name, seen[name])
            seen[name] += 1
            if key not in dur:
                order.append(key)
            dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{len(steps)} steps")
    tot = collections.defaultdict(float)
    for key in order:
        v = dur[key]
        m = sum(v) / len(v)
        tot[key[0]] += m
        print(f"{key[0]:64s} #{key[1]:2d}  {m:8.2f} us  (n {len(v)})")
    for name, t in tot.items():
        print(f"{name:64s} per step {t:9.1f} us")


if __name__ == "__main__":
    main()
