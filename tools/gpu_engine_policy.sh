#!/usr/bin/env bash
# Engine memory-policy A/B: parity tests per policy, then latency / concurrency.
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"; mkdir -p gpurun_out tools/_build
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_engine_policy.log 2>&1 || { tail -30 gpurun_out/pytest_engine_policy.log; exit 1; }
tail -1 gpurun_out/pytest_engine_policy.log
gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_concurrency
gcc -O2 -std=c99 -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
    -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/host_latency
{
for pol in 0 1 2; do
  echo "# policy $pol"
  HL_ENGINE=1 HL_ENGINE_POLICY=$pol timeout -k 10 100 tools/_build/host_latency | grep -E '"vec": (4096|8192),' | grep -E "Encode|lost=4|Update"
  HL_ENGINE=1 HL_ENGINE_POLICY=$pol timeout -k 10 100 tools/_build/host_concurrency 8192 300 131072 0 1 2 8 16 | grep threads
done
} > gpurun_out/engine_policy.log 2>&1
cut -c1-160 gpurun_out/engine_policy.log
