#!/bin/bash
# EDEN batch kernel times in three separate processes (placement dependence check).
set -e
O=$1; R=$PWD; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/p$i -o s --output-format csv -- python3 $R/tools/bench_eden.py > $R/$O/p$i.log 2>&1
done
echo eden prof done
