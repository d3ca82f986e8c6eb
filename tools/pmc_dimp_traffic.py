"""HBM traffic of the mfDiMP feature net per batch from rocprofv3 PMC passes (tools/pmc_dimp_traffic.sh) -> JSON
(committed under profiles/, read by bench.py's mfdimp_rgbt roofline as `traffic`).

FETCH_SIZE (doubled: gfx950 reports half the bytes of 16-B-per-lane streaming reads, MI355X_MICROARCH.md HBM
section) + WRITE_SIZE, KiB per dispatch, summed over the feature net's kernels (image normalisation, every conv and
split-K reduce, the InstanceL2Norm passes).  Dispatches are cut into feature-net passes at each normalize_kernel
(one per extract_backbone); only the passes at the largest grid (the 32-image batches of the timed steps, not the
tracker initialisation's) are averaged.  FETCH_SIZE counts the L2's fabric requests, Infinity-Cache hits included.

usage: python tools/pmc_dimp_traffic.py <pmc dir> <out.json> [algorithmic bytes per batch]"""
import csv
import glob
import json
import sys
from collections import defaultdict

root, out = sys.argv[1], sys.argv[2]
alg = float(sys.argv[3]) if len(sys.argv) > 3 else None
FEATURE = ("conv", "normalize", "maxpool", "l2norm")
rows = defaultdict(list)   # counter -> [(dispatch id, kernel, grid, value)]
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void mmt::", "").replace("mmt::", "").split("(mmt::")[0].split("(")[0]
        did = int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))
        rows[r["Counter_Name"]].append((did, k, int(r.get("Grid_Size", 0) or 0), float(r["Counter_Value"])))
res = {"algorithmic_bytes_per_batch": alg, "per_kernel_MB_per_batch": {}, "batches": {}}
per_kernel = defaultdict(float)
total = {}
for c, rs in rows.items():
    rs.sort()
    passes, cur = [], None
    for did, k, grid, v in rs:
        if k.startswith("normalize_kernel"):
            cur = {"grid": grid, "bytes": 0.0, "kern": defaultdict(float)}
            passes.append(cur)
        if cur is None or not k.startswith(FEATURE):
            continue
        b = v * 1024 * (2.0 if c == "FETCH_SIZE" else 1.0)
        cur["bytes"] += b
        cur["kern"][k] += b
    big = max(p["grid"] for p in passes)
    keep = [p for p in passes if p["grid"] == big]
    res["batches"][c] = len(keep)
    total[c] = sum(p["bytes"] for p in keep) / len(keep)
    for p in keep:
        for k, b in p["kern"].items():
            per_kernel[k] += b / len(keep)
fetch, write = total.get("FETCH_SIZE", 0.0), total.get("WRITE_SIZE", 0.0)
res.update({"bytes_per_batch": fetch + write, "fetch_bytes_per_batch": fetch, "write_bytes_per_batch": write,
            "ratio_to_algorithmic": (fetch + write) / alg if alg else None,
            "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of bench.py --workload "
                      "mfdimp_rgbt --sync (FETCH_SIZE x2 on gfx950); feature-net kernels of the 32-image passes"})
res["per_kernel_MB_per_batch"] = {k: round(v / 1e6, 2) for k, v in sorted(per_kernel.items(), key=lambda t: -t[1])}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: res[k] for k in ("bytes_per_batch", "fetch_bytes_per_batch", "write_bytes_per_batch",
                                      "ratio_to_algorithmic", "batches")}))
for k, v in list(res["per_kernel_MB_per_batch"].items())[:8]:
    print(f"  {k}: {v} MB")
