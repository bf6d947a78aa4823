#!/bin/bash
# round 5 profiling: biased torch-tie timeline, QUIC-FL batch (packed table on / off) with SQ and
# memory counters on the sender kernel, EDEN kernel stats
set -e
R=$PWD; O=$R/gpurun_out/r5e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_quicfl_sender.py tests/test_gpu_quicfl_c4.py tests/test_capi.py -m "gpu or not gpu" -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
for p in 1 0; do UQDME_QUICFL_PACKED=$p timeout -k 10 200 python tools/bench_quicfl.py --per-call 5 >> $O/quicfl_bench.jsonl; done
echo quicfl ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/biased_trace -o t --output-format csv -- python3 $R/tools/bench_biased.py --ties torch --steps 3 > $O/biased_trace.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/eden_stats -o s --output-format csv -- python3 $R/tools/bench_eden.py --steps 3 > $O/eden_stats.log 2>&1
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY" "FETCH_SIZE" "WRITE_SIZE"; do
  tag=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d $O/qfl_pmc_$tag -o p --output-format csv -- python3 $R/tools/bench_quicfl.py --steps 1 --per-call 0 > $O/qfl_pmc_$tag.log 2>&1
done
echo done
