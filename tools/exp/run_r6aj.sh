#!/bin/bash
# round 6 end-to-end regression, continued: C4 laplace and bernoulli on the final tree (their
# earlier runs: profiles/r6e_* and r6g_*; the laplace run drew the 21-point grid)
set -e
O=gpurun_out/r6aj; mkdir -p $O
timeout -k 10 900 python -u tools/nmse_curves.py --dim 4194304 --dists laplace --instances 50 --users 1,6,11,16,21,26,31,36,41,46,51,56,61,66,71,76,81,86,91,96,101 --schemes eden,unbiased,biased,quicfl --out $O/nmse_c4_laplace_i50.json > $O/laplace.log 2>&1
echo laplace ok
timeout -k 10 600 python -u tools/nmse_curves.py --dim 4194304 --dists bernoulli --instances 50 --schemes eden,unbiased,biased,quicfl --out $O/nmse_c4_bernoulli_i50.json > $O/bernoulli.log 2>&1
echo bernoulli ok
