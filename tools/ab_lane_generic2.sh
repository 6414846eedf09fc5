#!/usr/bin/env bash
# A/B: 8-byte (default) vs 16-byte lane units: 12+4 (fixed-column kernel),
# Update / Replace (accumulate kernels) and more generic 3-row shapes.
set -e
for km in "12 4" "10 4" "8 3" "16 3" "12 3"; do
  set -- $km
  echo "== $1+$2 encode / update / replace3"
  AB_K=$1 AB_M=$2 AB_ROUNDS=8 timeout -k 10 200 python -u tools/ab.py "" "lane_bytes=16" "op=upd" "op=upd,lane_bytes=16" "op=rep3" "op=rep3,lane_bytes=16"
done
