"""Per-kernel-class HBM traffic from tests/pmc_bench.sh output -> JSON (committed under profiles/).

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KiB per dispatch; on gfx950 FETCH_SIZE
reports half the bytes of 16-B-per-lane streaming reads (MI355X_MICROARCH.md, HBM section), so it is
doubled; WRITE_SIZE is taken as is.  Kernel classes are keyed by the kernel template signature."""
import csv
import glob
import json
import sys
from collections import defaultdict

root, out = sys.argv[1], sys.argv[2]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mmt::" not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].replace("void mmt::", "").replace("mmt::", "").split("(mmt::")[0].split("(float")[0]
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for name, cs in vals.items():
    d = {"dispatches": max(len(v) for v in cs.values())}
    if "FETCH_SIZE" in cs:
        d["fetch_bytes_per_dispatch"] = 2 * 1024 * sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
    if "WRITE_SIZE" in cs:
        d["write_bytes_per_dispatch"] = 1024 * sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
    if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
        h, m = sum(cs["TCC_HIT_sum"]), sum(cs["TCC_MISS_sum"])
        d["l2_hit_rate"] = h / max(h + m, 1)
    if "fetch_bytes_per_dispatch" in d and "write_bytes_per_dispatch" in d:
        d["traffic_bytes_per_dispatch"] = d["fetch_bytes_per_dispatch"] + d["write_bytes_per_dispatch"]
    res[name] = d
json.dump({"note": "FETCH_SIZE x2 (gfx950 16-B streaming-read correction) + WRITE_SIZE, KiB -> bytes; "
                   "means over all dispatches of the kernel class in a short bench.py run",
           "kernels": res}, open(out, "w"), indent=1)
for k, d in sorted(res.items(), key=lambda kv: -kv[1].get("traffic_bytes_per_dispatch", 0)):
    print(f"{k[:70]:70s} n={d['dispatches']:4d} traffic/dispatch {d.get('traffic_bytes_per_dispatch', 0) / 1e6:9.2f} MB"
          f"  L2 hit {d.get('l2_hit_rate', 0):.2f}")
