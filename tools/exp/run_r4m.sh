set -o pipefail
mkdir -p gpurun_out/r4m && export TMPDIR=/tmp
O=gpurun_out/r4m
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_quicfl.py tests/test_gpu_quicfl_sender.py > $O/gputests.log 2>&1; rc=$?; echo rc=$rc >> $O/gputests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 200 python -u tools/bench_quicfl.py --clients 1024 --dim 1048576 --bits 1 > $O/qfl.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_quicfl.py --clients 1024 --dim 1048576 --bits 4 >> $O/qfl.log 2>&1 || exit 1
echo done
