#!/bin/bash
# round 5: biased torch-tie chain with the one-wave LDS tail -- tests, stop / margin sweep, trace
set -e
R=$PWD; O=$R/gpurun_out/r5x; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_biased.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
echo tests ok
for cfg in "16384 2" "16384 3" "8192 2" "8192 3" "32768 2" "65536 2"; do
  set -- $cfg
  UQDME_TIE_STOP=$1 UQDME_TIE_MARGIN=$2 timeout -k 10 120 python tools/bench_biased.py --ties torch | sed "s/^{/{\"stop\": $1, \"margin\": $2, /" >> $O/sweep.jsonl
done
cd /tmp && export TMPDIR=/tmp
UQDME_TIE_STOP=16384 UQDME_TIE_MARGIN=2 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/bt -o t --output-format csv -- python3 $R/tools/bench_biased.py --ties torch --steps 3 > $O/bt.log 2>&1
echo done
