#!/bin/bash
# A/B of the libraries in _build/abl/ on the EDEN round trip at several batch shapes.
#   bash tools/exp/run_eden_shapes.sh <tag> ["n d" ...]
set -e
O=gpurun_out/${1:-r3zi}; shift
mkdir -p $O
SHAPES=("$@")
[ ${#SHAPES[@]} -eq 0 ] && SHAPES=("1024 1048576" "128 4194304" "1 4194304" "1024 172554")
for S in "${SHAPES[@]}"; do
  set -- $S
  EDEN_N=$1 EDEN_D=$2 timeout -k 10 240 python tools/exp/eden_variants.py > $O/eden_ab_$1_$2.jsonl 2> $O/eden_ab_$1_$2.err
done
echo done
