#!/usr/bin/env bash
# Same-box A/B of T concurrent 10+4 @ 8 KiB host Encode callers
# (tools/host_concurrency.c, every result checked) between the current
# library and another build (default tools/_build/r04prev), alternating.
# Output: gpurun_out/engine_conc_ab.log
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OTHER="${1:-tools/_build/r04prev}"
mkdir -p gpurun_out tools/_build
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -L"$OTHER" -lrsamd \
    -Wl,-rpath,"$PWD/$OTHER" -o tools/_build/host_concurrency_other
{
  for i in 1 2; do
    for v in host_concurrency host_concurrency_other; do
      echo "# $v pageable ($i)"
      timeout -k 10 200 tools/_build/$v 8192 300 131072 0 1 2 4 8 16 2>&1 | grep '^{"threads"'
      echo "# $v registered ($i)"
      timeout -k 10 200 env HL_REGISTER=1 tools/_build/$v 8192 300 131072 0 1 2 4 8 16 2>&1 | grep '^{"threads"'
    done
  done
} > gpurun_out/engine_conc_ab.log 2>&1
