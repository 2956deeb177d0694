#!/bin/bash
# Host-side AddressSanitizer + UBSan run of the CPU codec kernels
# (csrc/cpu_ops.cpp, csrc/sketch_hash.h) -- SURVEY.md §5.2.  GPU ASan is not
# available on this pool; the device kernels are covered by the fp32-reference
# numerics tests and the determinism tests instead.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-/tmp/commeff_sanitize}
mkdir -p "$OUT"
read -r TINC TLIB ABI < <(python - <<'PY'
import os, torch
r = os.path.dirname(torch.__file__)
print(os.path.join(r, "include"), os.path.join(r, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI))
PY
)
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
  -D_GLIBCXX_USE_CXX11_ABI=$ABI -I"$ROOT/commefficient_amd/csrc" -I"$TINC" \
  -I"$TINC/torch/csrc/api/include" \
  "$ROOT/tests/native/cpu_ops_harness.cpp" "$ROOT/commefficient_amd/csrc/cpu_ops.cpp" \
  -L"$TLIB" -Wl,-rpath,"$TLIB" -lc10 -ltorch_cpu -o "$OUT/cpu_ops_asan"
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$OUT/cpu_ops_asan"
