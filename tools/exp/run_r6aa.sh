#!/bin/bash
# round 6: the jump path's pass A on the side stream (KQ1ar) or in the runs, now that 1024
# messages take the jump path
set -e
O=gpurun_out/r6aa; mkdir -p $O
for r in 1 2; do for v in base noar; do
  for n in 1024 512 128; do
    timeout -k 10 120 python tools/exp/variants.py run $v -- tools/bench_quicfl.py --clients $n --per-call 0 --digest | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_quicfl_2p20.jsonl
  done
  timeout -k 10 180 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 4194304 quicfl | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_c4_quicfl.jsonl
done; done
echo ab ok
