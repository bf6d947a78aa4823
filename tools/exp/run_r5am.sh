#!/bin/bash
# round 5: KB6 part 1 after KB7a's first levels -- tests, then the heavy-level count sweep
set -e
O=gpurun_out/r5am; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_biased.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
echo tests ok
for rep in 1 2; do
for h in 0 1 2 3 4; do
  UQDME_TIE_HEAVY=$h timeout -k 10 120 python tools/bench_biased.py --ties torch | sed "s/^{/{\"heavy\": $h, /" >> $O/sweep.jsonl
done
done
echo done
