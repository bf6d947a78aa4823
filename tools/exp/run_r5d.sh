#!/bin/bash
# round 5: EDEN 1-bit fused norm + bins + dot; full bench
set -e
O=gpurun_out/r5d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_eden.py tests/test_gpu_dme.py tests/test_gpu_quicfl.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
for b in 1 2; do timeout -k 10 120 python tools/bench_eden.py --clients 1024 --bits $b >> $O/eden_bench.jsonl; done
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo done
