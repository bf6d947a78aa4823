set -e
R=$PWD; O=gpurun_out/r3k; mkdir -p $O
bash tools/round_check.sh r3k tests:test_gpu_eden.py tests:test_gpu_quicfl.py tests:test_gpu_dme.py tests:test_gpu_pipeline.py tests:test_gpu_parity.py bench
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $R/$O/bsq -o p --output-format csv -- python3 $R/tools/bench_biased.py --ties lowest --steps 2 > $R/$O/bsq.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/$O/bfetch -o p --output-format csv -- python3 $R/tools/bench_biased.py --ties lowest --steps 2 > $R/$O/bfetch.log 2>&1
echo r3k all done
