#!/bin/bash
# round 6 final check on one box: every -m gpu test, smoke, the bench (N=1 and the gloo self-launch
# with per_rank), per-call latencies, the round profile (kernel-trace stats + PMC passes), and
# kernel traces of the EDEN batch and the C4 shapes
set -e
bash tools/round_check.sh r6z tests smoke bench self2 dropin profile
O=gpurun_out/r6z
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/eden -o e --output-format csv -- python3 $R/tools/bench_eden.py --clients 1024 --bits 1 > $R/$O/eden_trace.log 2>&1
echo eden trace ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/c4 -o c --output-format csv -- python3 $R/tools/exp/c4_shapes.py 4194304 > $R/$O/c4_trace.log 2>&1
echo c4 trace ok
