#!/usr/bin/env bash
# A/B on the interleaved [S][d+p][len] layout: generic 3-4-row Encode on
# 16-byte units (default) vs 8-byte units (var=201).
set -e
for km in "16 4" "8 4" "6 3" "20 4"; do
  set -- $km
  echo "== $1+$2 encode, interleaved"
  AB_K=$1 AB_M=$2 AB_ROUNDS=8 timeout -k 10 200 python -u tools/ab.py "layout=inter" "var=201,layout=inter"
done
