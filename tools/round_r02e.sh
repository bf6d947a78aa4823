#!/bin/bash
# GPU box: all GPU tests, smoke, bench (with the output-placement probe), round profile.
set -e
O=gpurun_out/r02e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python bench.py --no-side-pipelines --no-cpu-baseline > $O/bench2.json 2> $O/bench2.err
bash tools/profile_round.sh $O/prof codes > $O/prof.log 2>&1
echo r02e done
