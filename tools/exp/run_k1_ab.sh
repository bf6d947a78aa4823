#!/bin/bash
# A/B of the libraries in _build/abl/: K1 alone and K1 + K2 (ablate.py), then L1 + biased (biased_variants.py).
set -e
O=gpurun_out/${1:-r05r}; mkdir -p $O
timeout -k 10 200 python tools/ablate.py run > $O/ablate_1.txt 2>&1
timeout -k 10 200 python tools/ablate.py run > $O/ablate_2.txt 2>&1
REPS=3 timeout -k 10 300 python tools/exp/biased_variants.py > $O/biased_variants.jsonl 2> $O/biased_variants.err
echo done
