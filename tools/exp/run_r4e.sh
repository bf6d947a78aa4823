set -o pipefail
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r4e_gputests.log 2>&1; rc=$?; echo rc=$rc >> gpurun_out/r4e_gputests.log
# test failures (rc 1) still let the measurements run; a time limit, abort or crash ends the call
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4e_smoke.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_quicfl.py --clients 1024 --dim 1048576 --bits 1 > gpurun_out/r4e_qfl.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/bench_quicfl.py --clients 16 --dim 4194304 --bits 2 >> gpurun_out/r4e_qfl.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/dropin_latency.py --dims 1024,2048,4096,32767,32768,172554,1048576,4194304 > gpurun_out/r4e_dropin.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/exp/oneshot_pool.py > gpurun_out/r4e_oneshot.log 2>&1 || exit 1
bash tools/pmc_sidepaths.sh gpurun_out/r4e_pmc > gpurun_out/r4e_pmc.log 2>&1 || exit 1
