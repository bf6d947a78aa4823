#!/bin/bash
# round 5: torch-tie replay with the LDS queue through ds_* accesses -- tests, phase timers, sweep
set -e
O=gpurun_out/r5z; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_biased.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1
echo tests ok
UQDME_TIE_STOP=16384 UQDME_TIE_MARGIN=2 timeout -k 10 120 python tools/exp/tie_prof.py run >> $O/prof.jsonl
for cfg in "16384 2" "16384 3" "8192 2" "8192 3" "32768 2" "65536 2"; do
  set -- $cfg
  UQDME_TIE_STOP=$1 UQDME_TIE_MARGIN=$2 timeout -k 10 120 python tools/bench_biased.py --ties torch | sed "s/^{/{\"stop\": $1, \"margin\": $2, /" >> $O/sweep.jsonl
done
echo done
