#!/bin/bash
# VGPR / scratch / spill report of every kernel in one csrc/*.hip file
# (device-only gfx950 compile; no GPU needed).  Usage: scripts/kernel_resources.sh conv
set -e
SRC=$(cd "$(dirname "$0")/.." && pwd)/commefficient_amd/csrc
OUT=$(mktemp /tmp/kres.XXXXXX.o)
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --offload-device-only --no-gpu-bundle-output \
  -c -I"$SRC" "$SRC/$1.hip" -o "$OUT"
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$OUT" |
  grep -E "^\s+\.name:|private_segment_fixed_size|\.vgpr_count|vgpr_spill" | paste - - - - |
  sed -E 's/ +/ /g; s/\.name: _ZN7commeff12_GLOBAL__N_1//'
rm -f "$OUT"
