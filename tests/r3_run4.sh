#!/bin/bash
# Round-3 GPU run 4: kernel trace of the mfDiMP bench (f16x3 convs, device tracker) at 32 sequences
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run4
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python bench.py --workload mfdimp_rgbt --batch 32 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1
cp $(find $O/prof -name '*kernel_stats.csv' | head -n 1) $O/kernel_stats.csv
python tests/prof_summary.py $O/kernel_stats.csv 12 40 > $O/summary.txt
python - <<'PY' > $O/conv_shapes.txt
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/r3_run4/prof/" + [f for f in __import__("os").listdir("gpurun_out/r3_run4/prof") if f.endswith("kernel_trace.csv")][0])))
by = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if "conv" in n:
        key = (n.split("(")[0][-40:], r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Grid_Size_Y", ""))
        by[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v)/1e3/12:9.1f} us/step  n={len(v):4d} avg {sum(v)/len(v)/1e3:7.1f} us  {k}")
PY
rm -rf $O/prof
