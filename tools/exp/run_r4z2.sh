set -o pipefail
mkdir -p gpurun_out/r4z2 && export TMPDIR=/tmp
O=gpurun_out/r4z2
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gputests.log 2>&1; rc=$?; echo rc=$rc >> $O/gputests.log
[ $rc = 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
echo done
