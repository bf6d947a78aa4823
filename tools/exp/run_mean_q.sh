#!/bin/bash
set -e
O=gpurun_out/${1:-r05k}; mkdir -p $O
timeout -k 10 200 python tools/exp/mean_q_variants.py > $O/mean_q.jsonl 2> $O/mean_q.err
echo done
