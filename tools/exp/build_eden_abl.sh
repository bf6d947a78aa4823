#!/bin/bash
# round 6: KE2+4 (eden_normdot1_kernel) variants into _build/abl/ for tools/exp/eden_variants.py:
# base, the pipelined norm chain, and three diagnostics (no dot waves / no bins stores / no chain)
set -e
cd "$(dirname "$0")/../.."
P=unbiased-quantization-distributed-mean-estimation_amd
A=$P/_build/abl; rm -rf $A; mkdir -p $A
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero"
O="$P/_build/uq_mt_poly.o $P/_build/uq_legacy_rng.o -lpthread"
for v in "a_base:" "b_pipe:-DUQ_EXP_CHAIN_PIPE" "c_nodot:-DUQ_EXP_NO_DOT" "d_nobins:-DUQ_EXP_NO_BINS" "e_nochain:-DUQ_EXP_NO_CHAIN"; do
  n=${v%%:*}; d=${v#*:}
  /opt/rocm/bin/hipcc $F $d -o $A/$n.so $P/csrc/uq_dme.hip -x none $O &
done
wait
ls $A
