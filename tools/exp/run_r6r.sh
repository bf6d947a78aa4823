#!/bin/bash
# round 6: QUIC-FL receiver runs at two waves per SIMD (up to 2048 run waves; the receiver
# kernels fit 2 waves without spills): digests and A/B
set -e
O=gpurun_out/r6r; mkdir -p $O
for r in 1 2; do for v in base r13 r18; do
  for n in 1024 768 512; do
    timeout -k 10 120 python tools/exp/variants.py run $v -- tools/bench_quicfl.py --clients $n --per-call 0 --digest | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_quicfl_2p20.jsonl
  done
  timeout -k 10 180 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 4194304 quicfl | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_c4_quicfl.jsonl
done; done
echo ab ok
