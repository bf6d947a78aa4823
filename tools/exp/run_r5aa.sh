#!/bin/bash
# round 5: kernel trace of the torch-tie batch (current build), for the replay kernel's duration
set -e
R=$PWD; O=$R/gpurun_out/r5aa; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
UQDME_TIE_STOP=${1:-16384} UQDME_TIE_MARGIN=${2:-2} timeout -k 10 200 rocprofv3 --kernel-trace -d $O/bt -o t --output-format csv -- python3 $R/tools/bench_biased.py --ties torch --steps 3 > $O/bt.log 2>&1
echo done
