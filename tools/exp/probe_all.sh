#!/bin/bash
# Placement probe over all 16 output sets, three bench processes (K2 per set + the timed K2).
set -e
O=gpurun_out/r05b; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-side-pipelines --probe-min 16 > $O/probe_all_$i.json 2> $O/probe_all_$i.err
done
echo done
