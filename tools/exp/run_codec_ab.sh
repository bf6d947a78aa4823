#!/bin/bash
set -e
O=gpurun_out/${1:-r05s}; mkdir -p $O
timeout -k 10 240 python tools/exp/codec_variants.py > $O/codec_ab.jsonl 2> $O/codec_ab.err
echo done
