#!/bin/bash
# round 6: harness + QUIC-FL tests after the legacy-draw rewrite, C4 shapes re-measured, and a
# 2-instance C4 normal curve to time the new draws against the GPU work
set -e
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dme.py tests/test_gpu_quicfl.py tests/test_gpu_quicfl_c4.py tests/test_gpu_quicfl_sender.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
timeout -k 10 300 python -u tools/exp/c4_shapes.py > $O/c4_shapes.jsonl 2> $O/c4_shapes.err
echo shapes ok
timeout -k 10 600 python -u tools/nmse_curves.py --dim 4194304 --dists normal --instances 2 --schemes eden,unbiased,biased,quicfl --out $O/nmse_normal_i2.json > $O/normal.log 2>&1
echo curves ok
