set -o pipefail
mkdir -p gpurun_out/r4g && export TMPDIR=/tmp
O=gpurun_out/r4g
timeout -k 10 600 python -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_quicfl.py tests/test_gpu_quicfl_sender.py tests/test_gpu_biased.py tests/test_gpu_dme.py > $O/gputests.log 2>&1; rc=$?; echo rc=$rc >> $O/gputests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 200 python -u tools/dropin_latency.py --dims 1024,2048,4096,32768,1048576,4194304 > $O/dropin.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_quicfl.py --clients 1024 --dim 1048576 --bits 1 > $O/qfl.log 2>&1 || exit 1
R=$PWD
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$O/bprof_4194304 -o s --output-format csv -- python3 $R/tools/dropin_prof.py 4194304 Type_biased_quantize > $R/$O/bprof.log 2>&1 || exit 1
echo done
