#!/usr/bin/env bash
# Host-side AddressSanitizer run of the C ABI (no GPU needed): librsamd with
# the host code instrumented (-Xarch_host -fsanitize=address; device code is
# untouched), then the strict-C99 consumer's host checks and the randomised
# host fuzzer.  Output in /tmp/rsamd_asan.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT=/tmp/rsamd_asan
mkdir -p "$OUT"
/opt/rocm/bin/hipcc -O1 -g -std=c++17 -fPIC -shared --offload-arch=gfx950 -fvisibility=hidden \
    -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -I "$ROOT/include" \
    "$ROOT"/reedsolomon_amd/csrc/{codec,host_calls,batches,host_batches,engine,watchdog,jit,jit_asm}.cpp \
    "$ROOT/reedsolomon_amd/csrc/kernels.hip" -o "$OUT/librsamd.so" -lhiprtc -lamd_comgr -ldl
for prog in tests/c/rs_consumer tools/host_fuzz; do
  /opt/rocm/llvm/bin/clang -std=c99 -O1 -g -fsanitize=address -I "$ROOT/include" "$ROOT/$prog.c" \
      -L"$OUT" -lrsamd -Wl,-rpath,"$OUT" -o "$OUT/$(basename "$prog")"
done
export ASAN_OPTIONS=detect_leaks=1:abort_on_error=1
"$OUT/rs_consumer" host
"$OUT/host_fuzz" "${1:-20000}"
