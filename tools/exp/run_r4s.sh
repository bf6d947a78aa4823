set -o pipefail
mkdir -p gpurun_out/r4s && export TMPDIR=/tmp
O=gpurun_out/r4s
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_quicfl.py tests/test_gpu_quicfl_sender.py tests/test_gpu_dme.py > $O/gputests.log 2>&1; rc=$?; echo rc=$rc >> $O/gputests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
for c in 128 256 1024; do timeout -k 10 200 python -u tools/bench_quicfl.py --clients $c --dim 1048576 --bits 1 --per-call 0 >> $O/qfl.log 2>&1 || exit 1; done
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
echo done
