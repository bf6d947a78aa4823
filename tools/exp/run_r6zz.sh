#!/bin/bash
# round 6 closing check on the final tree: every -m gpu test, smoke, the bench (N=1 and the gloo
# self-launch), the QUIC-FL / EDEN batch side lines
set -e
bash tools/round_check.sh r6zz tests smoke bench self2
O=gpurun_out/r6zz
timeout -k 10 200 python tools/bench_quicfl.py --clients 1024 > $O/quicfl_1024.json 2> $O/quicfl_1024.err
timeout -k 10 200 python tools/bench_eden.py --clients 1024 --bits 1 > $O/eden.json 2> $O/eden.err
echo side lines ok
