#!/bin/bash
# Build and run the native core stress test under AddressSanitizer+UBSan and
# ThreadSanitizer (host code only).  usage: scripts/sanitize_core.sh
set -eu
cd "$(dirname "$0")/.."
out=build/sanitize
mkdir -p $out
SRC="csrc/core/test_core.cpp csrc/core/membership.cpp csrc/core/wire.cpp csrc/core/ingest.cpp"
COMMON="-std=c++17 -g -O1 -fno-omit-frame-pointer -Icsrc/core -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lamdhip64 -lpthread"
g++ -fsanitize=address,undefined -fno-sanitize-recover=undefined $SRC -o $out/test_core_asan $COMMON
g++ -fsanitize=thread $SRC -o $out/test_core_tsan $COMMON
ASAN_OPTIONS=detect_leaks=1 $out/test_core_asan
TSAN_OPTIONS=halt_on_error=1 $out/test_core_tsan
