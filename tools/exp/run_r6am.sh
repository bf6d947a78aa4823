#!/bin/bash
# round 6: the unbiased kernels with 512-thread workgroups and 8192-element tiles (kQBlock 512):
# every -m gpu test on that build, then A/B against 256 at C4's shapes and the bench
set -e
O=gpurun_out/r6am; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
for r in 1 2; do for v in base new; do
  timeout -k 10 120 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 4194304 unbiased | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_c4_unbiased.jsonl
  timeout -k 10 120 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 1048576 unbiased | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_2p20_unbiased.jsonl
  timeout -k 10 200 python tools/exp/variants.py run $v -- bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-side-pipelines | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_bench.jsonl
done; done
echo ab ok
