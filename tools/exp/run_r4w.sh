set -o pipefail
mkdir -p gpurun_out/r4w && export TMPDIR=/tmp
O=gpurun_out/r4w
timeout -k 10 200 python -u tools/exp/biased_small_probe.py > $O/probe.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_biased.py > $O/gputests.log 2>&1; rc=$?; echo rc=$rc >> $O/gputests.log
exit $rc
