#!/bin/bash
# round 6: EDEN's segmented dot (KE4s) up to 128 clients: tests and A/B at C4's 101 x 2^22 and
# around the threshold at 2^20
set -e
O=gpurun_out/r6i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_eden.py tests/test_gpu_eden_norm.py tests/test_gpu_quicfl_c4.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
for r in 1 2; do for v in base new; do
  timeout -k 10 120 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 4194304 eden | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_c4_eden.jsonl
  for n in 65 100 128; do
    timeout -k 10 120 python tools/exp/variants.py run $v -- tools/bench_eden.py --clients $n --bits 1 | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_eden_2p20.jsonl
  done
done; done
echo ab ok
