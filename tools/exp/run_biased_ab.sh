#!/bin/bash
# A/B of two libraries in _build/abl/ (biased batch + L1), plain and under a kernel trace.
set -e
O=gpurun_out/${1:-r05i}; mkdir -p $O
REPS=3 timeout -k 10 240 python tools/exp/biased_variants.py > $O/biased_ab.jsonl 2> $O/biased_ab.err
R=$PWD; cd /tmp && export TMPDIR=/tmp
REPS=3 timeout -k 10 240 rocprofv3 --kernel-trace -d $R/$O/trace -o t --output-format csv -- python3 $R/tools/exp/biased_variants.py > $R/$O/biased_ab_trace.jsonl 2>&1
echo done
