#!/bin/bash
# round 5: biased batch with the fine first digit (KB6f lists the threshold bucket)
set -e
O=gpurun_out/r5c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_biased.py tests/test_gpu_large.py tests/test_gpu_dme.py tests/test_gpu_eden.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
for t in torch lowest; do timeout -k 10 200 python tools/bench_biased.py --ties $t >> $O/biased_bench.jsonl 2>> $O/biased_bench.err; done
timeout -k 10 200 python tools/bench_biased.py --ties torch --dist smallint >> $O/biased_bench.jsonl 2>> $O/biased_bench.err
echo bench ok
for b in 1 2; do timeout -k 10 120 python tools/bench_eden.py --clients 1024 --bits $b >> $O/eden_bench.jsonl; done
timeout -k 10 300 python tools/dropin_latency.py --dims 2048,172554,1048576,4194304 > $O/dropin.json
echo done
