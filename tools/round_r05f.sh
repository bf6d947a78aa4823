#!/bin/bash
# K1a four-wide ops: biased + parity GPU tests, then biased batch timings and a kernel-trace pass.
set -e
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_biased.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 120 python tools/bench_biased.py --ties lowest > $O/biased_lowest.json 2>&1
timeout -k 10 120 python tools/bench_biased.py --ties torch > $O/biased_torch.json 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/stats -o s --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_biased.py --ties torch > $GRAFT_REPO_ROOT/$O/stats.log 2>&1
echo r05f done
