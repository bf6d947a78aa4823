#!/bin/bash
# Time the K2 variants built by tools/exp/k2_variants.py, two processes.
set -e
O=gpurun_out/${1:-r05c}; mkdir -p $O
timeout -k 10 180 python tools/ablate.py run > $O/k2_variants_1.txt 2>&1
timeout -k 10 180 python tools/ablate.py run > $O/k2_variants_2.txt 2>&1
echo done
