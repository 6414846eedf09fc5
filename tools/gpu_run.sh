#!/usr/bin/env bash
# One parameterised GPU-box runner (replaces the per-pass gpu_r0*.sh scripts
# of rounds 1-2).  Each argument is one step; steps run in order, each under
# its own time limit, and the run stops at the first step that fails (no
# GPU step runs after a fault, abort or time-out).  Outputs go to
# gpurun_out/<tag>.log.
#
#   tools/gpu_run.sh smoke
#   tools/gpu_run.sh "tests:tests/test_gpu_tune_sweep.py"      # pytest -m gpu on those paths
#   tools/gpu_run.sh tests                                      # every GPU test
#   tools/gpu_run.sh bench "bench:--config 12+4@1MiB"           # bench.py (driver's command + extra args)
#   tools/gpu_run.sh "ops:--only wide"                          # tools/ops_bench.py with args
#   tools/gpu_run.sh "ab:AB_K=16,AB_M=16:op=rec16,jit=0:op=rec16,jit=2"   # tools/ab.py: env, then specs
#   tools/gpu_run.sh "py:tools/some_probe.py args"              # any python script
#   tools/gpu_run.sh "bin:tools/_build/valu_probe"              # a prebuilt probe binary
#   tools/gpu_run.sh "prof:<tag>:<python args>"                 # rocprofv3 kernel trace + stats of a python command
#   tools/gpu_run.sh "pmc:<tag>:<counters>:<python args>"       # one rocprofv3 --pmc pass (own run)
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="$REPO/gpurun_out"
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
n=0

fail() { echo "== step $n ($1) FAILED rc=$2; stopping"; tail -30 "$3"; exit 1; }

for step in "$@"; do
  n=$((n + 1))
  kind="${step%%:*}"
  arg=""
  [[ "$step" == *:* ]] && arg="${step#*:}"
  log="$OUT/step${n}_${kind}.log"
  echo "== step $n: $step"
  case "$kind" in
    smoke)
      timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 || fail "$step" $? "$log"
      tail -2 "$log" ;;
    tests)
      paths="${arg:-tests}"
      # shellcheck disable=SC2086
      timeout -k 10 1000 python -u -m pytest $paths -m gpu -x -v -l -p no:cacheprovider --timeout 300 \
          --timeout-method thread > "$log" 2>&1 || fail "$step" $? "$log"
      tail -3 "$log" ;;
    bench)
      # shellcheck disable=SC2086
      timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 $arg > "$log" 2>&1 || fail "$step" $? "$log"
      grep '^{' "$log" | cut -c1-400 ;;
    ops)
      # shellcheck disable=SC2086
      timeout -k 10 900 python -u tools/ops_bench.py $arg > "$log" 2>&1 || fail "$step" $? "$log"
      tail -40 "$log" ;;
    ab)
      envs="${arg%%:*}"
      specs="${arg#*:}"
      IFS=':' read -ra sp <<< "$specs"
      IFS=',' read -ra ev <<< "$envs"
      timeout -k 10 600 env "${ev[@]}" python -u tools/ab.py "${sp[@]}" > "$log" 2>&1 || fail "$step" $? "$log"
      cat "$log" ;;
    bin)
      # shellcheck disable=SC2086
      timeout -k 10 300 $arg > "$log" 2>&1 || fail "$step" $? "$log"
      tail -40 "$log" ;;
    py)
      # shellcheck disable=SC2086
      timeout -k 10 900 python -u $arg > "$log" 2>&1 || fail "$step" $? "$log"
      tail -40 "$log" ;;
    prof)
      tag="${arg%%:*}"
      cmd="${arg#*:}"
      export TMPDIR=/tmp
      # shellcheck disable=SC2086
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$tag" -o "$tag" -- python3 -u $cmd \
          > "$log" 2>&1 || fail "$step" $? "$log"
      tail -5 "$log" ;;
    pmc)
      tag="${arg%%:*}"
      rest="${arg#*:}"
      counters="${rest%%:*}"
      cmd="${rest#*:}"
      export TMPDIR=/tmp
      # shellcheck disable=SC2086
      timeout -s KILL 240 rocprofv3 --pmc $counters -f csv -d "$OUT/pmc_$tag" -o "$tag" -- python3 -u $cmd \
          > "$log" 2>&1 || fail "$step" $? "$log"
      tail -5 "$log" ;;
    *)
      echo "unknown step kind: $kind"; exit 2 ;;
  esac
done
echo "== all $n steps ok"
