#!/bin/bash
# round 6: QUIC-FL KQ1a (pass A on the side stream beside the sender's RHT and norm): tests and
# A/B of the 1024 x 2^20 batch; then any C4 curve left to finish (checkpoints in ckpt/)
set -e
O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_quicfl.py tests/test_gpu_quicfl_sender.py tests/test_gpu_quicfl_c4.py tests/test_gpu_dme.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
for r in 1 2; do for v in base new; do
  timeout -k 10 180 python tools/exp/variants.py run $v -- tools/bench_quicfl.py --clients 1024 --bits 1 --per-call 0 | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_quicfl.jsonl
done; done
for r in 1 2; do for k in narrow wide; do
  if [ $k = narrow ]; then export UQDME_K1B_NARROW=1; else unset UQDME_K1B_NARROW; fi
  timeout -k 10 120 python tools/exp/c4_shapes.py 4194304 unbiased | sed "s/^{/{\"k1b\": \"$k\", \"round\": $r, /" >> $O/ab_k1b_c4_unbiased.jsonl
done; done
unset UQDME_K1B_NARROW
echo ab ok
for dist in $CURVES; do
timeout -k 10 800 python -u tools/nmse_curves.py --dim 4194304 --dists $dist --instances 50 --schemes eden,unbiased,biased,quicfl --checkpoint $O/c4_{dist}.npz --resume-from ckpt/c4_{dist}.npz --time-limit 540 --out $O/nmse_c4_${dist}_i50.json > $O/$dist.log 2>&1
echo $dist ok
done
