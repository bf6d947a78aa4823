#!/bin/bash
# round 6: the placement lottery's second counter pass (DRAM-credit stalls and in-flight levels
# per TCC instance, fast vs slow set in one process), EDEN bins staged in LDS (tests + A/B), and
# the C4 laplace curve at 50 instances
set -e
O=gpurun_out/r6e; mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_DRAM_CREDIT_STALL TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_LEVEL TCC_EA0_RDREQ_LEVEL -d $R/$O/stall -o stall --output-format json -- python3 $R/tools/exp/placement_pmc.py 8 3 > $R/$O/stall.log 2>&1
echo pmc ok
cd $R
python tools/exp/placement_channels.py $O/stall/stall_results.json 3 $O/placement_channels_stalls.json > $O/placement_channels_stalls.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest tests/test_gpu_eden.py tests/test_gpu_eden_norm.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest_eden.log 2>&1
echo eden tests ok
for r in 1 2 3; do for v in base new; do
  timeout -k 10 120 python tools/exp/variants.py run $v -- tools/bench_eden.py --clients 1024 --bits 1 | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/ab_eden.jsonl
done; done
echo ab ok
timeout -k 10 900 python -u tools/nmse_curves.py --dim 4194304 --dists laplace --instances 50 --schemes eden,unbiased,biased,quicfl --checkpoint $O/c4_{dist}.npz --resume-from ckpt/c4_{dist}.npz --time-limit 600 --out $O/nmse_c4_laplace_i50.json > $O/laplace.log 2>&1
echo curves ok
