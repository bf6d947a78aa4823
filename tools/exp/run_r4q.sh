set -o pipefail
mkdir -p gpurun_out/r4q && export TMPDIR=/tmp
O=gpurun_out/r4q
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_quicfl_sender.py tests/test_gpu_quicfl.py tests/test_gpu_dme.py > $O/gputests.log 2>&1; rc=$?; echo rc=$rc >> $O/gputests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 200 python -u tools/bench_quicfl.py --clients 1024 --dim 1048576 --bits 1 --per-call 0 > $O/qfl.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_quicfl.py --clients 16 --dim 4194304 --bits 2 --per-call 0 >> $O/qfl.log 2>&1 || exit 1
R=$PWD; cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$O/stats -o s --output-format csv -- python3 $R/tools/bench_quicfl.py --clients 1024 --dim 1048576 --bits 1 --steps 2 --per-call 0 > $R/$O/stats.log 2>&1 || exit 1
echo done
