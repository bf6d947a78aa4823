#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter per rocprofv3 run, --kernel-trace only) over the
# biased and EDEN batches (1024 x 2^20) and the QUIC-FL sender, then per-kernel byte tables.
# usage (GPU box, repo root): tools/pmc_sidepaths.sh OUTDIR
set -e
R=$PWD; OUT=$R/$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for job in "biased:tools/bench_biased.py --clients 1024 --dim 1048576 --steps 3" \
           "eden:tools/bench_eden.py --clients 1024 --dim 1048576 --steps 3" \
           "quicfl:tools/bench_quicfl.py --clients 1024 --dim 1048576 --steps 2 --per-call 0"; do
  name=${job%%:*}; cmd=${job#*:}
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/$name/fetch -o p --output-format csv -- python3 $R/$cmd > $OUT/$name.fetch.log 2>&1
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/$name/write -o p --output-format csv -- python3 $R/$cmd > $OUT/$name.write.log 2>&1
done
echo done
