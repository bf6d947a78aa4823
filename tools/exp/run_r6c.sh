#!/bin/bash
# round 6: parity tests for the stream kernel's 3-tile prefetch and the EDEN bins-store order,
# A/B (HEAD vs tree) of both, then the first C4 curve at the reference's protocol (normal, 50
# instances, checkpointed)
set -e
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exact_scan.py tests/test_gpu_eden.py tests/test_gpu_eden_norm.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
for r in 1 2; do for v in base new; do
  timeout -k 10 120 python tools/exp/variants.py run $v -- tools/bench_eden.py --clients 1024 --bits 1 | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_eden.jsonl
  timeout -k 10 120 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 4194304 unbiased | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_c4_unbiased.jsonl
done; done
echo ab ok
timeout -k 10 900 python -u tools/nmse_curves.py --dim 4194304 --dists normal --instances 50 --schemes eden,unbiased,biased,quicfl --checkpoint $O/c4_{dist}.npz --resume-from ckpt/c4_{dist}.npz --time-limit 700 --out $O/nmse_c4_normal_i50.json > $O/normal.log 2>&1
echo curves ok
