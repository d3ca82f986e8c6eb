#!/bin/bash
# Round-3 GPU run 4: kernel trace of the mfDiMP bench (f16x3 convs, device tracker) at 32 sequences
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3_run4
mkdir -p $O
timeout -k 10 200 python bench.py --workload mfdimp_rgbt --batch 32 --steps 20 --warmup 3 --no-cpu-baseline --sync \
  > $O/bench_sync.json 2> $O/bench_sync.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python bench.py --workload mfdimp_rgbt --batch 32 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1
cp $(find $O/prof -name '*kernel_stats.csv' | head -n 1) $O/kernel_stats.csv
cp $(find $O/prof -name '*kernel_trace.csv' | head -n 1) $O/kernel_trace.csv
python tools/prof_summary.py $O/kernel_stats.csv 12 40 > $O/summary.txt
python - <<'PY' > $O/conv_shapes.txt
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/r3_run4/kernel_trace.csv")))
by = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    key = (n.split("(")[0][-48:], r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Grid_Size_Y", ""),
           r.get("Workgroup_Size_X", ""))
    by[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v)/1e3/12:9.1f} us/step  n={len(v):5d} avg {sum(v)/len(v)/1e3:8.2f} us  {k}")
PY
gzip -f $O/kernel_trace.csv
rm -rf $O/prof
