set -o pipefail
mkdir -p gpurun_out/r4h && export TMPDIR=/tmp
O=gpurun_out/r4h
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_biased.py > $O/gputests.log 2>&1; rc=$?; echo rc=$rc >> $O/gputests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 200 python -u tools/dropin_latency.py --dims 1024,2048,1048576,4194304 > $O/dropin.log 2>&1 || exit 1
timeout -k 10 1000 python -u tools/nmse_curves.py --dim 4194304 --instances 5 --users 1,6,11,51,101 --out $O/nmse_curves_d4194304.json > $O/nmse.log 2>&1 || exit 1
echo done
