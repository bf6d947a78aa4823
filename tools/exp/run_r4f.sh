set -o pipefail
mkdir -p gpurun_out/r4f && export TMPDIR=/tmp
O=gpurun_out/r4f
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gputests.log 2>&1; rc=$?; echo rc=$rc >> $O/gputests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 120 python -u tools/exp/oneshot_pool.py > $O/oneshot2.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/exp/oneshot_pool.py > $O/oneshot3.log 2>&1 || exit 1
R=$PWD
cd /tmp
for d in 1024 4194304; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$O/bprof_$d -o s --output-format csv -- python3 $R/tools/dropin_prof.py $d Type_biased_quantize > $R/$O/bprof_$d.log 2>&1 || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$O/qprof -o s --output-format csv -- python3 $R/tools/bench_quicfl.py --clients 1024 --dim 1048576 --bits 1 --steps 2 --per-call 0 > $R/$O/qprof.log 2>&1 || exit 1
echo done
