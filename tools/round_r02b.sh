#!/bin/bash
# GPU box: new GPU tests, round profile (stats + PMC), experiments, bench.  Each step has its own limit.
set -e
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_flower_hook.py tests/test_gpu_distributed.py -x -v --timeout 200 --timeout-method thread > $O/gputest_new.log 2>&1
timeout -k 10 120 python -u tools/exp/mall_groups.py > $O/mall_groups.jsonl 2> $O/mall_groups.err
timeout -k 10 120 python -u tools/exp/overlap.py > $O/overlap.jsonl 2> $O/overlap.err
bash tools/profile_round.sh $O/prof codes > $O/prof.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo r02b done
