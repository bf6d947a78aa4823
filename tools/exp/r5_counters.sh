#!/bin/bash
# Round-5 counter / trace pass (GPU box, repo root): bash tools/exp/r5_counters.sh OUTDIR
#  - FETCH_SIZE / WRITE_SIZE over the biased, EDEN and QUIC-FL batches (tools/pmc_sidepaths.sh)
#  - kernel-trace stats: biased torch-tie batch; QUIC-FL batch with the packed and the 8-byte table
#  - one SQ pass over the QUIC-FL batch (KQ1's issue / wait split)
set -e
R=$PWD; OUT=$R/$1; mkdir -p $OUT
bash tools/pmc_sidepaths.sh $1/bytes > $OUT/bytes.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/biased_trace -o s --output-format csv -- python3 $R/tools/bench_biased.py --clients 1024 --dim 1048576 --steps 3 > $OUT/biased_trace.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/qfl_packed -o s --output-format csv -- python3 $R/tools/bench_quicfl.py --clients 1024 --dim 1048576 --steps 3 --per-call 0 > $OUT/qfl_packed.log 2>&1
UQDME_QUICFL_PACKED=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/qfl_8b -o s --output-format csv -- python3 $R/tools/bench_quicfl.py --clients 1024 --dim 1048576 --steps 3 --per-call 0 > $OUT/qfl_8b.log 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d $OUT/qfl_sq -o p --output-format csv -- python3 $R/tools/bench_quicfl.py --clients 1024 --dim 1048576 --steps 2 --per-call 0 > $OUT/qfl_sq.log 2>&1
echo counters done
