#!/bin/bash
# round 5: list-strided key-digit passes -- tests, then torch / lowest A/B against HEAD
set -e
O=gpurun_out/r5av; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_biased.py tests/test_capi.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
echo tests ok
bash tools/exp/run_variants.sh $O 3 tools/bench_biased.py --ties torch
mv $O/variants.jsonl $O/variants_torch.jsonl
bash tools/exp/run_variants.sh $O 2 tools/bench_biased.py --ties lowest
mv $O/variants.jsonl $O/variants_lowest.jsonl
bash tools/exp/run_variants.sh $O 1 tools/bench_biased.py --ties torch --dist smallint
mv $O/variants.jsonl $O/variants_smallint.jsonl
echo done
