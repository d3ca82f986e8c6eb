#!/bin/bash
# Build a variant of libmmtrack.so with extra compile flags into abx/lib<name>.so (tuning A/Bs; MMTRACK_LIB selects it)
# usage: bash tools/build_variant.sh <name> "<-D flags>"
set -e
cd "$(dirname "$0")/../multi-modal-trakcing-bechmark_amd/csrc"
mkdir -p ../../abx
make -j8 -s OUT=../../abx/lib$1.so BUILD=/tmp/mmt_build_$1 \
  FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-value -I../../include $2"
