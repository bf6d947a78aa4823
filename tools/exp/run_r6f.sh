#!/bin/bash
# round 6: the small-batch K2 form with the tile prefix kernel (tests + A/B at C4 shapes), then
# the C4 gamma curve at 50 instances (checkpointed)
set -e
O=gpurun_out/r6f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exact_scan.py tests/test_gpu_pipeline.py tests/test_gpu_dme.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
for r in 1 2; do for v in base new; do
  timeout -k 10 120 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 4194304 unbiased | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_c4_unbiased.jsonl
done; done
echo ab ok
timeout -k 10 900 python -u tools/nmse_curves.py --dim 4194304 --dists gamma --instances 50 --schemes eden,unbiased,biased,quicfl --checkpoint $O/c4_{dist}.npz --resume-from ckpt/c4_{dist}.npz --time-limit 720 --out $O/nmse_c4_gamma_i50.json > $O/gamma.log 2>&1
echo curves ok
