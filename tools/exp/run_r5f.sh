#!/bin/bash
# round 5: config C4 NMSE curves (d = 2^22, 21 user counts, EDEN / unbiased / biased / QUIC-FL on
# the synthetic sender tables), normal and laplace in two processes side by side
set -e
O=$PWD/gpurun_out/r5f; mkdir -p $O
timeout -k 10 1100 python -u tools/nmse_curves.py --dim 4194304 --dists normal --instances 3 \
  --schemes eden,unbiased,biased,quicfl --out $O/nmse_curves_d4194304_normal.json > $O/normal.log 2>&1 &
P1=$!
timeout -k 10 1100 python -u tools/nmse_curves.py --dim 4194304 --dists laplace --instances 3 \
  --schemes eden,unbiased,biased,quicfl --out $O/nmse_curves_d4194304_laplace.json > $O/laplace.log 2>&1 &
P2=$!
R1=0; wait $P1 || R1=$?
R2=0; wait $P2 || R2=$?
echo "normal rc=$R1 laplace rc=$R2"
test $R1 -eq 0 -a $R2 -eq 0
