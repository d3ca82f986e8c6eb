#!/bin/bash
# Round 6 (second session), run 13 (second pass: the wait split into the tile's landing and the barrier): phase stamps of the 32-sequence attention kernel (attn_kernel<8, true>, ATTN_STAMPS
# build abx/libattnst.so): wave 0's cycles per key-tile loop part at N = 320 / 244 / 190 / 153, 16 and 32 sequences
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6_s2_run13
mkdir -p $O
MMTRACK_LIB=$PWD/abx/libattnst.so timeout -k 10 120 python tools/attn_stamps.py 32 320 244 190 153 > $O/stamps32.txt 2>&1 || { tail -5 $O/stamps32.txt; exit 1; }
MMTRACK_LIB=$PWD/abx/libattnst.so timeout -k 10 120 python tools/attn_stamps.py 16 320 > $O/stamps16.txt 2>&1 || { tail -5 $O/stamps16.txt; exit 1; }
python - <<'P'
import re, statistics
for f in ("gpurun_out/r6_s2_run13/stamps32.txt", "gpurun_out/r6_s2_run13/stamps16.txt"):
    cur, rows = None, {}
    for l in open(f):
        if l.startswith("## "):
            cur = l.strip()
            rows[cur] = []
        m = re.search(r"tiles (\d+): total (\d+) wait (\d+) s (\d+) softmax (\d+) pv (\d+) landed (\d+)", l)
        if m and cur:
            rows[cur].append([int(x) for x in m.groups()])
    for k, v in rows.items():
        if "launch 2" not in k or not v:
            continue
        med = [statistics.median(c) for c in zip(*v)]
        t = med[0]
        print(f"{k}: {len(v)} blocks, tiles {t:.0f}, per tile cycles: total {med[1] / t:.0f}, "
              f"S {med[3] / t:.0f}, softmax {med[4] / t:.0f}, PV {med[5] / t:.0f}, tile landed {med[6] / t:.0f}, "
              f"barrier + next issue {med[2] / t:.0f}")
P
