#!/bin/bash
# round 6 end-to-end regression: config C4 normal at the reference's protocol (50 instances, the
# driver's 21 user counts, EDEN / unbiased / biased / QUIC-FL) on the final tree; the curves
# must equal round 6's earlier run (profiles/r6c_nmse_curves_d4194304_normal_i50.json) exactly
set -e
O=gpurun_out/r6ai; mkdir -p $O
timeout -k 10 900 python -u tools/nmse_curves.py --dim 4194304 --dists normal --instances 50 --schemes eden,unbiased,biased,quicfl --out $O/nmse_c4_normal_i50.json > $O/normal.log 2>&1
echo c4 ok
