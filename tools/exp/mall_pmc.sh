#!/bin/bash
# FETCH_SIZE of K1 and K2 per step with groups of G clients, interleaved (K1(g) -> K2(g)) vs
# separate (all K1, then all K2).  usage (repo root, GPU box): bash tools/exp/mall_pmc.sh gpurun_out/<tag>
set -e
R=$PWD; OUT=$R/$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for G in 32 64 1024; do
  for I in 0 1; do
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/g${G}_i${I} -o p --output-format csv -- python3 $R/tools/exp/mall_groups.py --one $G $I 3 > $OUT/g${G}_i${I}.log 2>&1
  done
done
echo mall pmc done
