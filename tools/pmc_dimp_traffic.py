"""HBM traffic of the mfDiMP feature net per batch from rocprofv3 PMC passes (tools/pmc_dimp_traffic.sh) -> JSON
(committed under profiles/, read by bench.py's mfdimp_rgbt roofline as `traffic`).

FETCH_SIZE (doubled: gfx950 reports half the bytes of 16-B-per-lane streaming reads, MI355X_MICROARCH.md HBM
section) + WRITE_SIZE, KiB per dispatch, summed over the feature net's kernels (image normalisation, every conv and
split-K reduce, the max-pools, the InstanceL2Norm passes) and divided by the batches in the run -- one
extract_backbone + extract_classification_feat per tracked frame of the batch, counted by dimp_localize_kernel.

usage: python tools/pmc_dimp_traffic.py <pmc dir> <out.json> [algorithmic bytes per batch]"""
import csv
import glob
import json
import sys
from collections import defaultdict

root, out = sys.argv[1], sys.argv[2]
alg = float(sys.argv[3]) if len(sys.argv) > 3 else None
FEATURE = ("conv_", "normalize", "maxpool", "l2norm")
tot = defaultdict(float)
per_kernel = defaultdict(lambda: defaultdict(float))
batches = defaultdict(int)
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void mmt::", "").replace("mmt::", "").split("(mmt::")[0]
        c = r["Counter_Name"]
        if k.startswith("dimp_localize_kernel"):
            batches[c] += 1
        if not any(k.startswith(p) for p in FEATURE):
            continue
        v = float(r["Counter_Value"]) * 1024 * (2.0 if c == "FETCH_SIZE" else 1.0)
        tot[c] += v
        per_kernel[k.split("(")[0]][c] += v
n = {c: max(batches[c], 1) for c in tot}
fetch = tot["FETCH_SIZE"] / n["FETCH_SIZE"]
write = tot["WRITE_SIZE"] / n["WRITE_SIZE"]
res = {"bytes_per_batch": fetch + write, "fetch_bytes_per_batch": fetch, "write_bytes_per_batch": write,
       "batches": n, "algorithmic_bytes_per_batch": alg,
       "ratio_to_algorithmic": (fetch + write) / alg if alg else None,
       "per_kernel_MB_per_batch": {k: round(sum(v[c] / n[c] for c in v) / 1e6, 2) for k, v in per_kernel.items()},
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of bench.py --workload mfdimp_rgbt "
                 "--sync (FETCH_SIZE x2 on gfx950); feature-net kernels only"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: res[k] for k in ("bytes_per_batch", "fetch_bytes_per_batch", "write_bytes_per_batch",
                                      "ratio_to_algorithmic")}))
