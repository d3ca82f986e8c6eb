"""Per-kernel and per-class HBM traffic from tools/pmc_bench.sh output -> JSON (committed under profiles/).

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KiB per dispatch; on gfx950 FETCH_SIZE
reports half the bytes of 16-B-per-lane streaming reads (MI355X_MICROARCH.md, HBM section), so it is
doubled; WRITE_SIZE is taken as is.

Classes (the names bench.py's timing probe uses): the run is made with the two-stream halves off
(MMT_OVERLAP_MIN=0, as the probe runs), so each step's dispatches are in the engine's layer order and a
GEMM's class follows from its epilogue template argument -- 0 qkv, 1 fc1, 2 alternately proj then fc2
(every layer issues proj before fc2), 4 / 6 patch, 3 / 5 conv1 (head) -- and attn_kernel is attn.

usage: python tools/pmc_traffic.py <pmc dir> <out.json>"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

root, out = sys.argv[1], sys.argv[2]


def short(name):
    return name.replace("void mmt::", "").replace("mmt::", "").split("(mmt::")[0].split("(float")[0]


def epi_of(name):
    m = re.match(r"(gemm\w*_kernel)<([^>]*)>", name)
    if not m:
        return None
    args = [a.strip() for a in m.group(2).split(",")]
    if m.group(1) in ("gemm256s_kernel", "gemm256_kernel", "gemm128w_kernel"):
        return int(args[0])
    if m.group(1) == "gemm_kernel":
        return int(args[4])
    return int(args[4]) if len(args) > 4 else None   # persist / ring: <BM, BN, WMW, WNW, EPI, ...>


per_counter = defaultdict(list)      # counter -> [(dispatch id, kernel, value)]
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "mmt::" not in r["Kernel_Name"]:
            continue
        did = int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))
        per_counter[r["Counter_Name"]].append((did, short(r["Kernel_Name"]), float(r["Counter_Value"])))

kern = defaultdict(lambda: defaultdict(list))
cls = defaultdict(lambda: defaultdict(list))
for cname, rows in per_counter.items():
    rows.sort()
    resid_seen = 0
    for did, k, v in rows:
        kern[k][cname].append(v)
        e = epi_of(k)
        c = None
        if k.startswith("attn_kernel"):
            c = "attn"
        elif e == 0:
            c = "qkv"
        elif e == 1:
            c = "fc1"
        elif e == 2:
            c = "proj" if resid_seen % 2 == 0 else "fc2"
            resid_seen += 1
        elif e in (4, 6):
            c = "patch"
        elif e in (3, 5):
            c = "conv1"
        if c:
            cls[c][cname].append(v)


def summarise(cs):
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
    return d


res = {k: summarise(v) for k, v in kern.items()}
cres = {k: summarise(v) for k, v in cls.items()}
json.dump({"note": "FETCH_SIZE x2 (gfx950 16-B streaming-read correction) + WRITE_SIZE, KiB -> bytes; means over "
                   "all dispatches of the kernel / class in a short bench.py run with the two-stream halves off "
                   "(the timing probe's launch shapes); classes assigned by epilogue and layer order",
           "kernels": res, "classes": cres}, open(out, "w"), indent=1)
for k, d in sorted(cres.items(), key=lambda kv: -kv[1].get("traffic_bytes_per_dispatch", 0)):
    print(f"class {k:8s} n={d['dispatches']:4d} traffic/dispatch {d.get('traffic_bytes_per_dispatch', 0) / 1e6:9.2f} MB"
          f"  L2 hit {d.get('l2_hit_rate', 0):.2f}")
for k, d in sorted(res.items(), key=lambda kv: -kv[1].get("traffic_bytes_per_dispatch", 0)):
    print(f"{k[:70]:70s} n={d['dispatches']:4d} traffic/dispatch {d.get('traffic_bytes_per_dispatch', 0) / 1e6:9.2f} MB"
          f"  L2 hit {d.get('l2_hit_rate', 0):.2f}")
