#!/bin/bash
set -e
O=gpurun_out/${1:-r05d}; mkdir -p $O
timeout -k 10 240 python tools/exp/lane_bw.py > $O/lane_bw.jsonl 2> $O/lane_bw.err
echo done
