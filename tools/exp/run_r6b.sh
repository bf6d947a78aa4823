#!/bin/bash
# round 6: harness tests (checkpoint/resume), EDEN KE2+4 variants A/B, the gloo bench rehearsal
# with per_rank, and a 3-instance C4 normal run on the pipelined draws
set -e
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dme.py tests/test_gpu_quicfl_c4.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
timeout -k 10 240 python tools/exp/eden_variants.py > $O/eden_ab.jsonl 2> $O/eden_ab.err
echo eden ab ok
UQDME_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --no-side-pipelines --probe-candidates 4 --probe-min 4 > $O/bench_gloo2.json 2> $O/bench_gloo2.err
echo gloo ok
timeout -k 10 600 python -u tools/nmse_curves.py --dim 4194304 --dists normal --instances 3 --schemes eden,unbiased,biased,quicfl --out $O/nmse_normal_i3.json > $O/normal.log 2>&1
echo curves ok
