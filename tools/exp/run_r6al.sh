#!/bin/bash
# round 6: the C4 harness with every scheme's estimate queued before the host NMSE norms: the tests, then
# C4 bernoulli (host-bound) and normal (draw-bound) against their earlier curves and run times
set -e
O=gpurun_out/r6al; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dme.py tests/test_gpu_quicfl_c4.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
timeout -k 10 600 python -u tools/nmse_curves.py --dim 4194304 --dists bernoulli --instances 50 --schemes eden,unbiased,biased,quicfl --out $O/nmse_c4_bernoulli_i50.json > $O/bernoulli.log 2>&1
echo bernoulli ok
timeout -k 10 600 python -u tools/nmse_curves.py --dim 4194304 --dists normal --instances 50 --schemes eden,unbiased,biased,quicfl --out $O/nmse_c4_normal_i50.json > $O/normal.log 2>&1
echo normal ok
