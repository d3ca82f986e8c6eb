"""Per-step kernel breakdown of a rocprofv3 kernel trace over the steady-state steps of a bench run.

usage: python tools/trace_steps.py TRACE.csv[.gz] MARKER_KERNEL SKIP_STEPS [TOP]
A step starts at each launch of MARKER_KERNEL (e.g. dimp_sample_kernel or geometry_kernel); the first
SKIP_STEPS steps (warm-up / initialisation) and the last (partial) one are dropped."""
import collections
import csv
import gzip
import sys


def main():
    path, marker, skip = sys.argv[1], sys.argv[2], int(sys.argv[3])
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
    rows = list(csv.DictReader(gzip.open(path, "rt") if path.endswith(".gz") else open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    a, b = idx[skip], idx[-1]
    nst = len(idx) - 1 - skip
    sub = rows[a:b]
    t0, t1 = int(sub[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    busy, last = 0, t0
    for r in sub:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e > last:
            busy += e - max(s, last)
            last = e
    print(f"{nst} steps: wall/step {(t1 - t0) / 1e3 / nst:.1f} us, GPU busy/step {busy / 1e3 / nst:.1f} us, "
          f"launches/step {len(sub) / nst:.1f}")
    by = collections.defaultdict(list)
    for r in sub:
        n = r["Kernel_Name"].split("(")[0][-44:]
        by[(n, r.get("Grid_Size_X", ""), r.get("Grid_Size_Y", ""), r.get("Grid_Size_Z", ""))].append(
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = 0
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:top]:
        tot += sum(v)
        print(f"{sum(v) / 1e3 / nst:8.1f} us/step  n/step {len(v) / nst:5.1f}  avg {sum(v) / len(v) / 1e3:7.2f} us  {k}")


if __name__ == "__main__":
    main()
