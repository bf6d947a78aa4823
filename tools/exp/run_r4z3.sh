set -o pipefail
mkdir -p gpurun_out/r4z3 && export TMPDIR=/tmp
O=gpurun_out/r4z3
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_biased.py > $O/gputests.log 2>&1; rc=$?; echo rc=$rc >> $O/gputests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u tools/dropin_latency.py --dims 1024,2048,4096,32767,32768 > $O/dropin.log 2>&1 || exit 1
echo done
