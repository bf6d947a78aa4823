#!/bin/bash
# One GPU-box round check (replaces the per-round round_r0*.sh drivers of rounds 1-2).
#   bash tools/round_check.sh <tag> [steps...]      (run from the repo root on the GPU box)
# steps (default: tests smoke bench gloo2):
#   tests       all -m gpu tests               -> gpurun_out/<tag>/gputest.log
#   tests:<f>   only tests/<f> (repeatable, e.g. tests:test_gpu_pipeline.py)
#   smoke       __graft_entry__.smoke()       -> smoke.log
#   bench       python bench.py               -> bench.json
#   gloo2       2-rank gloo rehearsal of bench.py --gpus 2 under torch.distributed.run (ranks share cuda:0)
#   self2       the same, bench.py --gpus 2 starting its own ranks (no external launcher)
#   dropin      tools/dropin_latency.py       -> dropin_latency.json
#   profile     tools/profile_round.sh (kernel-trace stats + PMC passes, codes pipeline)
# Every GPU step runs under its own timeout and the first failure ends the call (set -e).
set -e
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
STEPS=${@:-tests smoke bench gloo2}
TESTS=""
for s in $STEPS; do case $s in tests:*) TESTS="$TESTS tests/${s#tests:}";; esac; done
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputest.log 2>&1 ;;
    tests:*) if [ -n "$TESTS" ]; then
               timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputest_sel.log 2>&1
               TESTS=""
             fi ;;
    smoke) timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 ;;
    bench) timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err ;;
    gloo2) UQDME_BENCH_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
             --master-addr 127.0.0.1 --master-port 29553 bench.py --gpus 2 --steps 5 --warmup 2 \
             > $O/bench_gloo2.json 2> $O/bench_gloo2.err ;;
    self2) UQDME_BENCH_BACKEND=gloo timeout -k 10 240 python bench.py --gpus 2 --steps 5 --warmup 2 \
             > $O/bench_self2.json 2> $O/bench_self2.err ;;
    dropin) timeout -k 10 200 python tools/dropin_latency.py > $O/dropin_latency.json 2> $O/dropin_latency.err ;;
    profile) bash tools/profile_round.sh $O codes4 > $O/profile.log 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  echo "$TAG: $s ok"
done
echo "$TAG done"
