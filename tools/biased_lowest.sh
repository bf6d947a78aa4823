#!/bin/bash
# GPU box: biased GPU tests, bench_biased with the lowest-index rule and torch ties, kernel profile.
set -e
O=$1; mkdir -p $O; R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gpu_biased.py -x -v --timeout 250 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 200 python tools/bench_biased.py > $O/bench_biased.log 2>&1
timeout -k 10 200 python tools/bench_biased.py --ties lowest >> $O/bench_biased.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o s --output-format csv -- python3 $R/tools/bench_biased.py --ties lowest > $R/$O/prof.log 2>&1
echo biased lowest done
