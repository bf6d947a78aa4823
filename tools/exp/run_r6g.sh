#!/bin/bash
# round 6: the WIDE K1b finalize (tests: L1 bits, large sizes, scan forms, biased, harness; A/B at
# C4 shapes), then the C4 bernoulli and lognormal curves at 50 instances (checkpointed)
set -e
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exact_scan.py tests/test_gpu_biased.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
for r in 1 2; do for v in base new; do
  timeout -k 10 120 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 4194304 unbiased,biased | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_c4.jsonl
done; done
echo ab ok
for dist in bernoulli lognormal; do
timeout -k 10 800 python -u tools/nmse_curves.py --dim 4194304 --dists $dist --instances 50 --schemes eden,unbiased,biased,quicfl --checkpoint $O/c4_{dist}.npz --resume-from ckpt/c4_{dist}.npz --time-limit 480 --out $O/nmse_c4_${dist}_i50.json > $O/$dist.log 2>&1
echo $dist ok
done
