#!/bin/bash
# round 6: the small-batch unbiased form's tile sums and maps in one pass (tile_summap_kernel,
# decoupled look-back): every -m gpu test, then A/B at C4's shapes and the per-call drop-in
set -e
O=gpurun_out/r6o; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
for r in 1 2; do for v in base new; do
  timeout -k 10 120 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 4194304 unbiased | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_c4_unbiased.jsonl
  timeout -k 10 120 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 1048576 unbiased | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_2p20_unbiased.jsonl
done; done
echo ab ok
