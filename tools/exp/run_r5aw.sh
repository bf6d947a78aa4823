#!/bin/bash
# round 5: y extent of the list-strided KB6 (UQDME_OUTPUT_GY) against HEAD, both tie rules
set -e
O=gpurun_out/r5aw; mkdir -p $O
for rep in 1 2; do
  for t in torch lowest; do
    for gy in 64 256 1024; do
      UQDME_OUTPUT_GY=$gy timeout -k 10 120 python tools/bench_biased.py --ties $t | sed "s/^{/{\"gy\": $gy, /" >> $O/sweep.jsonl
    done
    timeout -k 10 120 python tools/exp/variants.py run head -- tools/bench_biased.py --ties $t | sed "s/^{/{\"gy\": \"head\", /" >> $O/sweep.jsonl
  done
done
echo done
