set -o pipefail
mkdir -p gpurun_out/r4o && export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r4o
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $O/sq -o p --output-format csv -- python3 $R/tools/bench_quicfl.py --clients 1024 --dim 1048576 --bits 1 --steps 1 --per-call 0 > $O/sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU -d $O/sq2 -o p --output-format csv -- python3 $R/tools/bench_quicfl.py --clients 1024 --dim 1048576 --bits 1 --steps 1 --per-call 0 > $O/sq2.log 2>&1 || exit 1
echo done
