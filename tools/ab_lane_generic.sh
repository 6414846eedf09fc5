#!/usr/bin/env bash
# A/B: 8-byte (default) vs 16-byte lane units on the generic (runtime-column)
# one-chunk kernels, <= 4 output rows (tools/ab.py).
set -e
for km in "8 4" "6 3" "16 4" "20 4" "8 2" "4 2"; do
  set -- $km
  echo "== $1+$2 encode / reconst"
  AB_K=$1 AB_M=$2 AB_ROUNDS=8 timeout -k 10 200 python -u tools/ab.py "" "lane_bytes=16" "op=rec1" "op=rec1,lane_bytes=16"
done
