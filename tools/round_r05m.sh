#!/bin/bash
# GPU box: all GPU tests, smoke, bench (after the K3 and EDEN-norm non-temporal loads).
set -e
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo r05m done
