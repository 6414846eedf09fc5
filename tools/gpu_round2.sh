#!/usr/bin/env bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
echo "== pytest -m gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
echo "== ops bench"; timeout -k 10 600 python -u tools/ops_bench.py > $OUT/ops_bench.log 2>&1 || { tail -30 $OUT/ops_bench.log; exit 1; }
cat $OUT/ops_bench.log | grep -v amdgpu.ids
echo "== 2-rank rehearsal (gloo, both ranks on cuda:0)"
RSAMD_BENCH_BACKEND=gloo RSAMD_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 10 > $OUT/bench_2rank.log 2>&1 || { tail -30 $OUT/bench_2rank.log; exit 1; }
grep '^{' $OUT/bench_2rank.log | cut -c1-400
