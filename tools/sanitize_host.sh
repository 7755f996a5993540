#!/bin/bash
# Host-side sanitizer runs of the native CPU runtime (csrc/engine + the host/device headers):
# AddressSanitizer + UndefinedBehaviorSanitizer, then ThreadSanitizer for the threaded batch loops.
# (GPU ASan / xnack+ builds are not available on the target pool; device code is covered by the
# numerics tests against the CPU engines instead.)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${TMPDIR:-/tmp}/svoc_sanitize
mkdir -p "$OUT"
SRC=("$R/csrc/selftest/engine_selftest.cpp" "$R/csrc/engine/reference_cpu.cpp" "$R/csrc/engine/svoc_io.cpp")
INC=(-I"$R/csrc/include" -I"$R/csrc/engine")
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
    "${INC[@]}" "${SRC[@]}" -o "$OUT/selftest_asan" -pthread
ASAN_OPTIONS=detect_leaks=1 UBSAN_OPTIONS=print_stacktrace=1 "$OUT/selftest_asan" 8
g++ -std=c++17 -O1 -g -fsanitize=thread "${INC[@]}" "${SRC[@]}" -o "$OUT/selftest_tsan" -pthread
TSAN_OPTIONS=halt_on_error=1 "$OUT/selftest_tsan" 8
echo "sanitizers OK"
