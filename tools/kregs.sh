#!/bin/bash
# Per-kernel register / scratch use of one HIP source for gfx950 (device-only assembly, no GPU):
#   tools/kregs.sh csrc/file.hip [kernel-name regex] [extra hipcc flags...]
src=$1; pat=${2:-.}; shift 2
out=/tmp/kregs_$$.s
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$(dirname $0)/../include --cuda-device-only -S "$src" -o $out "$@" 2>/dev/null || exit 1
awk '/\.type.*@function/ {split($2, a, ","); name=a[1]} /^; NumVgprs:/ {v=$3} /^; NumAgprs:/ {ag=$3} /^; ScratchSize:/ {s=$3} /^; Occupancy:/ {print name, "vgpr", v, "agpr", ag, "scratch", s, "occ", $3}' $out | c++filt | grep -E "$pat" | cut -c1-220
rm -f $out
