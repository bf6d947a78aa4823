#!/bin/bash
# GPU box: all GPU tests, smoke, bench, then the round profile (kernel-trace stats + PMC passes).
set -e
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
UQDME_BENCH_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29553 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_gloo2.json 2> $O/bench_gloo2.err
bash tools/profile_round.sh $O codes
echo r05t done
