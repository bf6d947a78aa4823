#!/bin/bash
# round 6: QUIC-FL's receiver inverse RHT at D = 2^22 as 14 + 8 bits (fwht_low16k_kernel<0>):
# tests and A/B at C4's shapes
set -e
O=gpurun_out/r6j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_quicfl.py tests/test_gpu_quicfl_c4.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
for r in 1 2; do for v in base new; do
  timeout -k 10 180 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 4194304 quicfl | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_c4_quicfl.jsonl
done; done
echo ab ok
