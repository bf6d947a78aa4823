#!/bin/bash
# round 6: SQ counters of the QUIC-FL 1024 x 2^20 batch (VALU per message of the two-wave runs)
set -e
O=gpurun_out/r6ag; mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU -d $R/$O/sq1 -o p --output-format csv -- python3 $R/tools/bench_quicfl.py --clients 1024 --steps 1 --per-call 0 > $R/$O/sq1.log 2>&1
echo sq1 ok
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d $R/$O/sq2 -o p --output-format csv -- python3 $R/tools/bench_quicfl.py --clients 1024 --steps 1 --per-call 0 > $R/$O/sq2.log 2>&1
echo sq2 ok
