#!/bin/bash
# GPU box: SQ counters for the codec kernels (one pass each), for tools/pmc_table.py.
# usage (repo root): bash tools/codec_pmc.sh gpurun_out/<tag>
set -e
O=$1; R=$PWD; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $R/$O/sq1 -o p --output-format csv -- python3 $R/tools/codec_bench.py --steps 2 > $R/$O/sq1.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM -d $R/$O/sq2 -o p --output-format csv -- python3 $R/tools/codec_bench.py --steps 2 > $R/$O/sq2.log 2>&1
echo codec pmc done
