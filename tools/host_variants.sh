#!/usr/bin/env bash
# tools/host_latency.c Encode across vector sizes for each variant given as
# "label|VAR=value VAR=value" (host_latency's HL_* environment), in order.
# Every call's result is checked.  Output: gpurun_out/host_variants.log
#   tools/host_variants.sh "engine 8 wg|HL_REGISTER=1" "engine 64 wg|HL_REGISTER=1 HL_ENGINE_WAVES=64"
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out tools/_build
gcc -O2 -std=c99 -pthread -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_latency
{
  for v in "$@"; do
    label="${v%%|*}"; envs="${v#*|}"
    echo "# $label"
    # shellcheck disable=SC2086
    timeout -k 10 200 env HL_OPS="${HL_OPS:-1}" $envs tools/_build/host_latency 2>&1 | grep -v '^host_latency:'
  done
} > gpurun_out/host_variants.log 2>&1
