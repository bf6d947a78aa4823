#!/bin/bash
# round 6: QUIC-FL's jump-path runs at two waves per SIMD (launch bound 2 waves/EU, n*R up to
# 2048, the jump path up to 1024 messages): outputs digested per variant, A/B timings
set -e
O=gpurun_out/r6k; mkdir -p $O
for r in 1 2; do for v in base w2only w2 w1cap; do
  for n in 1024 512 256 128; do
    timeout -k 10 120 python tools/exp/variants.py run $v -- tools/bench_quicfl.py --clients $n --per-call 0 --digest | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_quicfl_2p20.jsonl
  done
  timeout -k 10 180 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 4194304 quicfl | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_c4_quicfl.jsonl
done; done
echo ab ok
# EDEN KE4 (one wave per client) with 32 loads in flight per lane instead of 16
for r in 1 2; do for v in base ke4u32; do
  timeout -k 10 180 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 4194304 eden | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_c4_eden.jsonl
  timeout -k 10 120 python tools/exp/variants.py run $v -- tools/bench_eden.py --clients 1024 --bits 2 | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_eden_2bit.jsonl
done; done
echo eden ok
