#!/bin/bash
# round 5: biased torch-tie chain -- KB7a stop / level margin sweep (1024-thread tails)
set -e
O=gpurun_out/r5v; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_biased.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
echo tests ok
for cfg in "65536 1" "65536 0" "65536 2" "32768 1" "131072 1" "16384 1"; do
  set -- $cfg
  for rep in 1 2; do
    UQDME_TIE_STOP=$1 UQDME_TIE_MARGIN=$2 timeout -k 10 120 python tools/bench_biased.py --ties torch | sed "s/^{/{\"stop\": $1, \"margin\": $2, /" >> $O/sweep.jsonl
  done
done
timeout -k 10 120 python tools/bench_biased.py --ties lowest >> $O/sweep.jsonl
echo done
