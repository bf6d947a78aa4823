#!/bin/bash
# round 6: K2 placement lottery by counter: TCC_EA0_WRREQ / _RDREQ over the
# C2 batch's K2 on the fastest and the slowest of 8 output sets, in one process; raw outputs in
# csv and json to see whether the per-TCC-instance values are kept.  Then the K2 stream forms
# at C4 shapes under a kernel trace.
set -e
O=gpurun_out/r6d; mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ TCC_EA0_RDREQ -d $R/$O/raw -o raw --output-format csv json -- python3 $R/tools/exp/placement_pmc.py 8 3 > $R/$O/raw.log 2>&1
echo pmc ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/c4trace -o c4 --output-format csv -- python3 $R/tools/exp/c4_shapes.py 4194304 unbiased > $R/$O/c4trace.log 2>&1
echo trace ok
