#!/bin/bash
# Round profile on the GPU box: kernel-trace stats + separate PMC passes.
# usage (repo root): bash tools/profile_round.sh gpurun_out/<tag> [pipeline: q|codes|codes4|encode]
# then: PROFILE_STEPS=40 python tools/summarize_profile.py gpurun_out/<tag> <tag> <pipeline>
set -e
PIPE=${2:-codes}
R=$PWD; OUT=$R/$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o s --output-format csv -- python3 $R/bench.py --steps 40 --warmup 2 --no-cpu-baseline --no-side-pipelines --pipeline $PIPE > $OUT/stats.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch -o p --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side-pipelines --pipeline $PIPE > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/write -o p --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side-pipelines --pipeline $PIPE > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $OUT/sq -o p --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side-pipelines --pipeline $PIPE > $OUT/sq.log 2>&1
echo profile done
