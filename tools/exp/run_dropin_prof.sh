#!/bin/bash
# Per-call drop-in: latency (host included) and a kernel trace of 30 calls per scheme and d.
#   bash tools/exp/run_dropin_prof.sh <tag> [schemes...]
set -e
O=gpurun_out/${1:-r05u}; shift
mkdir -p $O
SCHEMES=${@:-Type_unbiased_quantize}
timeout -k 10 200 python tools/dropin_latency.py > $O/dropin_latency.json 2> $O/dropin_latency.err
R=$PWD; cd /tmp && export TMPDIR=/tmp
for S in $SCHEMES; do
  for D in ${DIMS:-1048576 4194304}; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$O/prof_${S}_$D -o s --output-format csv -- python3 $R/tools/dropin_prof.py $D $S > $R/$O/prof_${S}_$D.log 2>&1
  done
done
echo done
