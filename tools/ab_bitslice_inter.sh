#!/usr/bin/env bash
# A/B on the interleaved [S][d+p][len] layout: bit-sliced (default) vs
# perm-table (bitslice=0) Encode.
set -e
for km in "10 8" "10 6" "12 8" "8 5"; do
  set -- $km
  echo "== $1+$2 encode, interleaved"
  AB_K=$1 AB_M=$2 AB_ROUNDS=8 timeout -k 10 200 python -u tools/ab.py "layout=inter" "bitslice=0,layout=inter"
done
