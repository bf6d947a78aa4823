set -o pipefail
mkdir -p gpurun_out/r4n && export TMPDIR=/tmp
O=gpurun_out/r4n
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_quicfl_sender.py tests/test_gpu_quicfl.py > $O/gputests.log 2>&1; rc=$?; echo rc=$rc >> $O/gputests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 200 python -u tools/bench_quicfl.py --clients 1024 --dim 1048576 --bits 1 --per-call 0 > $O/qfl.log 2>&1 || exit 1
echo done
