#!/usr/bin/env bash
# The one host-call runner (replaces round 4's engine_*.sh, host_sizes.sh,
# host_variants.sh, host_concurrency.sh and gpu_engine_sweep.sh).  Builds
# tools/host_latency.c and tools/host_concurrency.c against the current
# library (and, with OTHER=<dir of another librsamd.so>, against that one
# too, for a same-box A/B), then runs each spec in order:
#
#   lat|<label>|<ENV=v ...>                 one call's latency per size / op (host_latency)
#   conc|<label>|<ENV=v ...>|<args>         T concurrent callers (host_concurrency: vec reps co_max mixed T...)
#   lat-other|... / conc-other|...          the same against $OTHER
#
# ENV is host_latency's HL_* environment (HL_VEC, HL_SIZES, HL_OPS,
# HL_REGISTER, HL_GAP_US, HL_TUNE="knob=v,..." for any rs_tune knob, ...).
# Every call's result is checked by the tools.  Output: gpurun_out/<tag>.log
# (tag = $HP_TAG, default host_paths).  Examples:
#   tools/host_paths.sh "lat|8 KiB pageable|HL_VEC=8192" "lat|8 KiB registered|HL_VEC=8192 HL_REGISTER=1"
#   tools/host_paths.sh "lat|3 ms gaps|HL_VEC=8192 HL_GAP_US=3000" "conc|8 KiB|HL_REGISTER=1|8192 300 131072 0 1 8"
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out tools/_build
for t in host_latency host_concurrency; do
  gcc -O2 -std=c99 -pthread -Iinclude tools/$t.c -Lreedsolomon_amd/_lib -lrsamd \
      -Wl,-rpath,"$PWD/reedsolomon_amd/_lib" -o tools/_build/$t
  if [[ -n "${OTHER:-}" ]]; then
    gcc -O2 -std=c99 -pthread -Iinclude tools/$t.c -L"$OTHER" -lrsamd -Wl,-rpath,"$(cd "$OTHER" && pwd)" \
        -o tools/_build/${t}_other
  fi
done
LOG="gpurun_out/${HP_TAG:-host_paths}.log"
: > "$LOG"
for spec in "$@"; do
  IFS='|' read -r kind label envs args <<< "$spec"
  case "$kind" in
    lat) bin=tools/_build/host_latency ;;
    lat-other) bin=tools/_build/host_latency_other ;;
    conc) bin=tools/_build/host_concurrency ;;
    conc-other) bin=tools/_build/host_concurrency_other ;;
    *) echo "unknown spec kind: $kind" >&2; exit 2 ;;
  esac
  echo "# $kind: $label" | tee -a "$LOG"
  # shellcheck disable=SC2086
  timeout -k 10 300 env $envs $bin $args >> "$LOG" 2>&1
done
grep -v '^host_' "$LOG" | cut -c1-220
