#!/bin/bash
# round 5: KB7a stop / margin sweep on the current build (one box, alternated)
set -e
O=gpurun_out/r5al; mkdir -p $O
for rep in 1 2; do
for cfg in "16384 3" "16384 2" "8192 2" "8192 3" "16384 1"; do
  set -- $cfg
  UQDME_TIE_STOP=$1 UQDME_TIE_MARGIN=$2 timeout -k 10 120 python tools/bench_biased.py --ties torch | sed "s/^{/{\"stop\": $1, \"margin\": $2, /" >> $O/sweep.jsonl
done
done
timeout -k 10 120 python tools/bench_biased.py --ties lowest >> $O/sweep.jsonl
echo done
