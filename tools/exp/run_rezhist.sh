#!/bin/bash
set -e
O=gpurun_out/${1:-r05e}; mkdir -p $O
timeout -k 10 200 python tools/exp/rezhist_bw.py > $O/rezhist_bw.jsonl 2> $O/rezhist_bw.err
echo done
