#!/usr/bin/env bash
# A/B: the bit-sliced kernel on the 4-parity BASELINE shapes (bitslice=2)
# against the perm-table kernels (default), split and interleaved layouts.
set -e
for km in "10 4" "12 4"; do
  set -- $km
  echo "== $1+$2 encode"
  AB_K=$1 AB_M=$2 AB_ROUNDS=10 timeout -k 10 200 python -u tools/ab.py "" "bitslice=2" "layout=inter" "bitslice=2,layout=inter"
done
echo "== 10+4 encode, 8 KiB"
AB_VEC=8192 AB_ROUNDS=10 timeout -k 10 200 python -u tools/ab.py "" "bitslice=2"
