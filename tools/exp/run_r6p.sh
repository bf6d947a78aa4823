#!/bin/bash
# round 6: tile_summap_kernel issue order (tile-major vs client-major) against round 5's kernels
set -e
O=gpurun_out/r6p; mkdir -p $O
R=$PWD
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact_scan.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
for r in 1 2; do for v in base tm cm; do
  timeout -k 10 120 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 4194304 unbiased | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_c4_unbiased.jsonl
  timeout -k 10 120 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 1048576 unbiased | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_2p20_unbiased.jsonl
done; done
echo ab ok
cd /tmp && export TMPDIR=/tmp
for v in base tm; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/tr_$v -o t --output-format csv -- python3 $R/tools/exp/variants.py run $v -- $R/tools/exp/c4_shapes.py 4194304 unbiased > $R/$O/trace_$v.log 2>&1
done
echo trace ok
