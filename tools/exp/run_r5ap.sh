#!/bin/bash
# round 5: int32 workgroup partition (biased A/B vs HEAD) and the pair-table nibble mean (bench A/B)
set -e
O=gpurun_out/r5ap; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_biased.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
echo tests ok
bash tools/exp/run_variants.sh $O 3 tools/bench_biased.py --ties torch
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-side-pipelines | sed "s/^{/{\"variant\": \"pairtab\", /" >> $O/bench.jsonl
  timeout -k 10 300 python tools/exp/variants.py run base -- bench.py --no-cpu-baseline --no-side-pipelines | sed "s/^{/{\"variant\": \"nibtab16\", /" >> $O/bench.jsonl
done
echo done
