#!/bin/bash
# round 6: kernel traces of the QUIC-FL batch at 512 and 1024 messages (receiver per-round cost)
set -e
O=gpurun_out/r6v; mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp
for n in 512 1024; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/tr_$n -o t --output-format csv -- python3 $R/tools/bench_quicfl.py --clients $n --per-call 0 --steps 2 > $R/$O/trace_$n.log 2>&1
done
echo trace ok
