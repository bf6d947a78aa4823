#!/bin/bash
set -e
O=gpurun_out/${1:-r05g}; mkdir -p $O
REPS=${REPS:-2} timeout -k 10 300 python tools/exp/biased_variants.py > $O/biased_variants.jsonl 2> $O/biased_variants.err
echo done
