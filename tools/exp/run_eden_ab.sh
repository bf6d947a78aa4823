#!/bin/bash
# A/B of the libraries in _build/abl/ on the EDEN round trip, plain and under a kernel trace.
set -e
O=gpurun_out/${1:-r05l}; mkdir -p $O
timeout -k 10 240 python tools/exp/eden_variants.py > $O/eden_ab.jsonl 2> $O/eden_ab.err
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d $R/$O/trace -o t --output-format csv -- python3 $R/tools/exp/eden_variants.py > $R/$O/eden_ab_trace.jsonl 2>&1
echo done
