#!/bin/bash
# round 6: with the counting passes gone, the jump path at 1024 messages (two runs per message,
# two waves per SIMD) against the one-wave kernels: cost-model factors 1.8 (base) / 1.3 / 1.0
set -e
O=gpurun_out/r6x; mkdir -p $O
for r in 1 2; do for v in base s13 s13r13 s10r10; do
  for n in 1024 768 640; do
    timeout -k 10 120 python tools/exp/variants.py run $v -- tools/bench_quicfl.py --clients $n --per-call 0 --digest | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_quicfl_2p20.jsonl
  done
  timeout -k 10 180 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 4194304 quicfl | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_c4_quicfl.jsonl
done; done
echo ab ok
