#!/bin/bash
# round 6: kernel traces of the biased quantizer at C4's few-client shapes (6 and 101 x 2^22)
set -e
O=gpurun_out/r6ac; mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp
for n in 6 101; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/tr_$n -o t --output-format csv -- python3 $R/tools/bench_biased.py --clients $n --dim 4194304 --steps 3 > $R/$O/trace_$n.log 2>&1
done
echo trace ok
