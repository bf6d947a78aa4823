#!/bin/bash
# GPU box: codec GPU tests, codec bench (R = 1, 2), one kernel-trace profile.
# usage (repo root): bash tools/codec_check.sh gpurun_out/<tag>
set -e
O=$1; mkdir -p $O; R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -x -v --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 200 python tools/codec_bench.py > $O/codec_bench.jsonl 2>$O/codec_bench.err
timeout -k 10 200 python tools/codec_bench.py --bits 2 >> $O/codec_bench.jsonl 2>>$O/codec_bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o s --output-format csv -- python3 $R/tools/codec_bench.py > $R/$O/prof.log 2>&1
echo codec check done
