#!/bin/bash
# round 6: small-batch segmented stream with at most one wave of workgroups (no tail round)
set -e
O=gpurun_out/r6q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact_scan.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
for r in 1 2; do for v in base new; do
  timeout -k 10 120 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 4194304 unbiased | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_c4_unbiased.jsonl
  timeout -k 10 120 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 1048576 unbiased | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_2p20_unbiased.jsonl
done; done
echo ab ok
