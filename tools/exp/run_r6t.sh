#!/bin/bash
# round 6: lean (single-buffered) pass B in the two-wave runs kernel: 185 VGPRs, no spills;
# the cost model's two-wave factor 1.8 / 1.3 / 1.0 (1.0 takes R = 2 at 1024 messages)
set -e
O=gpurun_out/r6t; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_quicfl_sender.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
for r in 1 2; do for v in base lean lean_f10 lean_f13 lean3_f10 lean3_f15; do
  for n in 1024 512 384; do
    timeout -k 10 120 python tools/exp/variants.py run $v -- tools/bench_quicfl.py --clients $n --per-call 0 --digest | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_quicfl_2p20.jsonl
  done
  timeout -k 10 180 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 4194304 quicfl | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_c4_quicfl.jsonl
done; done
echo ab ok
