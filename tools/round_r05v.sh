#!/bin/bash
# GPU box: all GPU tests, smoke, per-call drop-in latency (after dropping the drop-in's input clone).
set -e
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python tools/dropin_latency.py > $O/dropin_latency.json 2> $O/dropin_latency.err
echo r05v done
