#!/bin/bash
# round 6: QUIC-FL jump path without the sender's counting pass over rot (runs write exact
# values into their own spans, KQ1f compacts) and with 16-byte mask loads in the receiver's count
set -e
O=gpurun_out/r6w; mkdir -p $O
R=$PWD
timeout -k 10 600 python -u -m pytest tests/test_gpu_quicfl_sender.py tests/test_gpu_quicfl.py tests/test_gpu_quicfl_c4.py tests/test_gpu_dme.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
echo tests ok
for r in 1 2; do for v in base new; do
  for n in 1024 512 384 128; do
    timeout -k 10 120 python tools/exp/variants.py run $v -- tools/bench_quicfl.py --clients $n --per-call 0 --digest | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_quicfl_2p20.jsonl
  done
  timeout -k 10 180 python tools/exp/variants.py run $v -- tools/exp/c4_shapes.py 4194304 quicfl | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_c4_quicfl.jsonl
done; done
echo ab ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/tr_512 -o t --output-format csv -- python3 $R/tools/bench_quicfl.py --clients 512 --per-call 0 --steps 2 > $R/$O/trace_512.log 2>&1
echo trace ok
