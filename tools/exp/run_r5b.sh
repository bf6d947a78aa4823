#!/bin/bash
# round 5: EDEN (MKL-order dot + bins kernel), QUIC-FL at 2^22 and the fused drop-in
set -e
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_eden.py tests/test_gpu_eden_norm.py tests/test_gpu_quicfl_c4.py tests/test_gpu_quicfl_sender.py tests/test_gpu_dme.py tests/test_gpu_paths_agree.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
for b in 1 2; do timeout -k 10 120 python tools/bench_eden.py --clients 1024 --bits $b >> $O/eden_bench.jsonl; done
echo eden ok
timeout -k 10 300 python tools/dropin_latency.py --quicfl --dims 2048,172554,1048576,4194304 > $O/dropin.json
echo done
