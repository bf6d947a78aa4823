#!/bin/bash
# round 5: biased torch-tie chain -- traces at two KB7a stops, and a wider sweep
set -e
R=$PWD; O=$R/gpurun_out/r5w; mkdir -p $O
for cfg in "65536 2" "16384 2" "16384 3" "8192 2" "32768 2" "65536 3"; do
  set -- $cfg
  UQDME_TIE_STOP=$1 UQDME_TIE_MARGIN=$2 timeout -k 10 120 python tools/bench_biased.py --ties torch | sed "s/^{/{\"stop\": $1, \"margin\": $2, /" >> $O/sweep.jsonl
done
cd /tmp && export TMPDIR=/tmp
for cfg in "65536 2" "16384 2"; do
  set -- $cfg
  UQDME_TIE_STOP=$1 UQDME_TIE_MARGIN=$2 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/bt_$1 -o t --output-format csv -- python3 $R/tools/bench_biased.py --ties torch --steps 3 > $O/bt_$1.log 2>&1
done
echo done
