#!/usr/bin/env bash
# Round-2 GPU pass ar: the multi-rank bench paths on the 1-GPU box (both ranks
# on cuda:0, gloo): under torch.distributed.run as the driver launches it, and
# `bench.py --gpus 2` starting its own ranks.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"; mkdir -p "$OUT"
RSAMD_BENCH_BACKEND=gloo RSAMD_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 20 --warmup 5 --cpu-seconds 2 > $OUT/ar_2rank_torchrun.log 2>&1 || { echo "rc $?"; tail -20 $OUT/ar_2rank_torchrun.log; exit 1; }
grep '^{' $OUT/ar_2rank_torchrun.log | cut -c1-330
RSAMD_BENCH_BACKEND=gloo RSAMD_BENCH_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --cpu-seconds 2 > $OUT/ar_2rank_spawn.log 2>&1 || { echo "rc $?"; tail -20 $OUT/ar_2rank_spawn.log; exit 1; }
grep '^{' $OUT/ar_2rank_spawn.log | cut -c1-330
