#!/bin/bash
# TLB counters of K2 (q + codes) in several processes (fast / slow mode), one PMC pass each.
R=$PWD; OUT=$R/$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for i in 1 2 3 4 5; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_THRASHING_STALL_sum -d $OUT/p$i -o p --output-format csv -- python3 $R/tools/exp/k2_once.py > $OUT/p$i.log 2>&1 || exit 1
done
echo done
