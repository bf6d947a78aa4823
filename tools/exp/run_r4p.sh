set -o pipefail
mkdir -p gpurun_out/r4p && export TMPDIR=/tmp
O=gpurun_out/r4p
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_quicfl.py tests/test_gpu_quicfl_sender.py tests/test_gpu_eden.py tests/test_gpu_dme.py > $O/gputests.log 2>&1; rc=$?; echo rc=$rc >> $O/gputests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 200 python -u tools/exp/qfl_dropin_breakdown.py > $O/bd.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/dropin_latency.py --quicfl --dims 1024,2048,1048576,4194304 > $O/dropin.log 2>&1 || exit 1
echo done
