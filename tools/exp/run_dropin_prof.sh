#!/bin/bash
# Per-call drop-in: latency (host included) and a kernel trace of 30 calls at d = 2^20 and 172 554.
set -e
O=gpurun_out/${1:-r05u}; mkdir -p $O
timeout -k 10 200 python tools/dropin_latency.py > $O/dropin_latency.json 2> $O/dropin_latency.err
R=$PWD; cd /tmp && export TMPDIR=/tmp
for D in 1048576 172554; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$D -o s --output-format csv -- python3 $R/tools/dropin_prof.py $D > $R/$O/prof_$D.log 2>&1
done
echo done
