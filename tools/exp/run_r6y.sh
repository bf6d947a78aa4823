#!/bin/bash
# round 6 final check (after the QUIC-FL / unbiased small-batch changes): every -m gpu test,
# smoke, the bench (N=1 and the gloo self-launch), per-call latencies, the round profile, clean
# C4 shapes, kernel traces of the EDEN and QUIC-FL batches and the C4 shapes
set -e
bash tools/round_check.sh r6y tests smoke bench self2 dropin profile
O=gpurun_out/r6y
R=$PWD
timeout -k 10 300 python tools/exp/c4_shapes.py 4194304 > $O/c4_shapes.jsonl 2> $O/c4_shapes.err
echo c4 clean ok
for n in 1024 512; do
  timeout -k 10 200 python tools/bench_quicfl.py --clients $n > $O/quicfl_$n.json 2> $O/quicfl_$n.err
done
timeout -k 10 200 python tools/bench_eden.py --clients 1024 --bits 1 > $O/eden.json 2> $O/eden.err
echo side lines ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/eden -o e --output-format csv -- python3 $R/tools/bench_eden.py --clients 1024 --bits 1 > $R/$O/eden_trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/qfl -o q --output-format csv -- python3 $R/tools/bench_quicfl.py --clients 1024 --per-call 0 --steps 2 > $R/$O/qfl_trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/c4 -o c --output-format csv -- python3 $R/tools/exp/c4_shapes.py 4194304 > $R/$O/c4_trace.log 2>&1
echo traces ok
