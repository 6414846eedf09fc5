#!/usr/bin/env bash
# Launch-parameter sweep of the encode bench (one process per setting).
# RSAMD_VAR=... experiments need RSAMD_LIB_VARIANT=experiments in the spec
# (librsamd_exp.so, `python -m reedsolomon_amd.build --experiments`): the
# product library ignores RSAMD_VAR.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG="${CFG:-10+4@1MiB}"
run() {
  local tag="$1"; shift
  local line
  line=$(env "$@" timeout -k 10 300 python -u bench.py --config "$CFG" --cpu-seconds 0 2>/dev/null | tail -1)
  local rc=$?
  python3 - "$tag" "$line" <<'PY'
import json, sys
tag, line = sys.argv[1], sys.argv[2]
try:
    j = json.loads(line)
    print(f"{tag:40s} value={j['value']:8.1f} GiB/s  kernel={j['roofline']['kernel_ms_mean']:.4f} ms  frac={j['roofline']['frac']:.3f}")
except Exception:
    print(f"{tag:40s} FAILED: {line[:200]}")
PY
  return $rc
}
for spec in "$@"; do
  # spec: tag:VAR=val,VAR=val
  tag="${spec%%:*}"; vars="${spec#*:}"
  IFS=',' read -ra kv <<< "$vars"
  run "$tag" "${kv[@]}" || exit 1
done
