#!/bin/bash
set -e
O=gpurun_out/r02k; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_codes.py tests/test_gpu_exact_scan.py -x -v --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
echo r02k done
